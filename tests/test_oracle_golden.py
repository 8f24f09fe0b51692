"""Pin the CPU oracle (and the host-side quant/pack restatements) to the golden fixtures.

The fixtures come from the reference's own Python (quant_minmax, quant.py:40-84) run in the build
container by tests/golden/make_golden.py; expected GroupGEMM outputs there are computed by an
independent numpy restatement, so these tests check the C oracle against a second implementation
of the same reference formulas (quantize.cuh:425-475, mm_tile.cuh:469-496, 610-662).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from mxmoe_amd.quantize import pack_wxax, quant_rtn_sym, unpack_wxax
from oracle import oracle

GOLD = Path(__file__).resolve().parent / "golden"


def _problems(name):
    d = np.load(GOLD / name)
    for i in range(int(d["P"])):
        M, N, K = (int(x) for x in d[f"p{i}_shape"])
        yield i, M, N, K, int(d[f"p{i}_bits"]), d


@pytest.mark.parametrize("bits", [8, 4])
def test_quant_matches_reference_quant_minmax(bits):
    d = np.load(GOLD / "quant_golden.npz")
    x, q_ref, s_ref = d[f"x_{bits}"], d[f"q_{bits}"], d[f"scale_{bits}"]
    q_o, s_o = oracle.quant_rtn_sym(x, bits)
    assert (s_o.view(np.uint16) == s_ref.view(np.uint16)).all()
    assert (q_o == q_ref).all()
    q_t, s_t = quant_rtn_sym(torch.from_numpy(x), bits)
    assert (s_t.numpy().view(np.uint16) == s_ref.view(np.uint16)).all()
    assert (q_t.numpy() == q_ref).all()


@pytest.mark.parametrize("name", ["gg_w8a8_small.npz", "gg_w4a4_small.npz", "gg_mixed_small.npz"])
def test_pack_matches_golden(name):
    for i, M, N, K, bits, d in _problems(name):
        if bits == 16:
            continue
        assert (oracle.pack_wxax(d[f"p{i}_qa"], bits) == d[f"p{i}_A"]).all()
        assert (pack_wxax(torch.from_numpy(d[f"p{i}_qb"]), bits).numpy() == d[f"p{i}_B"]).all()
        assert (oracle.unpack_wxax(d[f"p{i}_B"], bits, K) == d[f"p{i}_qb"]).all()
        assert (unpack_wxax(torch.from_numpy(d[f"p{i}_A"]), bits, K).numpy() == d[f"p{i}_qa"]).all()


@pytest.mark.parametrize("name", ["gg_w8a8_small.npz", "gg_w4a4_small.npz", "gg_mixed_small.npz"])
def test_oracle_gg_quant_bit_exact(name):
    for i, M, N, K, bits, d in _problems(name):
        if bits == 16:
            continue
        C = oracle.gg_quant(d[f"p{i}_A"], d[f"p{i}_B"], d[f"p{i}_sa"], d[f"p{i}_sb"], M, N, K, bits)
        assert (C.view(np.uint16) == d[f"p{i}_C"].view(np.uint16)).all(), f"problem {i}"
        assert (oracle.acc_exact(d[f"p{i}_qa"], d[f"p{i}_qb"]) == d[f"p{i}_acc"]).all()


def test_oracle_reproduces_reference_column_scale_bug_when_fed_permuted_scales():
    # "reference-as-written" (mm_tile.cuh:452,462-463) == intended arithmetic with sb'[c] = sb[f(c)]
    from tests.golden.make_golden import ref_bug_cols

    for i, M, N, K, bits, d in _problems("gg_w8a8_small.npz"):
        sbp = d[f"p{i}_sb"][ref_bug_cols(N)]
        C = oracle.gg_quant(d[f"p{i}_A"], d[f"p{i}_B"], d[f"p{i}_sa"], sbp, M, N, K, bits)
        assert (C.view(np.uint16) == d[f"p{i}_C_refbug"].view(np.uint16)).all()


def test_oracle_fp16_close_to_f64():
    for i, M, N, K, bits, d in _problems("gg_fp16_small.npz"):
        C = oracle.gg_f16(d[f"p{i}_A"], d[f"p{i}_B"], M, N, K).astype(np.float64)
        ref = d[f"p{i}_C_f64"]
        # output rounding to fp16 only: |err| <= 2^-11 |ref| (+ subnormal floor)
        assert (np.abs(C - ref) <= np.abs(ref) * 2.0 ** -11 + 2.0 ** -24).all()


def test_f16_conversions_round_trip_all_halves():
    lib = oracle.lib()
    for h in range(0, 1 << 16, 7):
        if (h & 0x7C00) == 0x7C00 and (h & 0x3FF):
            continue  # NaN payloads
        f = lib.oracle_f16_to_f32(h)
        assert np.float16(f).view(np.uint16) == h
        assert lib.oracle_f32_to_f16(f) == h


def test_f32_to_f16_rounding_matches_numpy():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 10.0 ** rng.integers(-9, 5, 20000),
                        np.float32([6.1035156e-05, 2.9802322e-08, 65519.0, 65520.0, -0.0, 5.9604645e-08])])
    lib = oracle.lib()
    got = np.array([lib.oracle_f32_to_f16(float(v)) for v in x.astype(np.float32)], dtype=np.uint16)
    assert (got == x.astype(np.float16).view(np.uint16)).all()


@pytest.mark.parametrize("bits", [8, 4])
def test_exhaustive_restatement_matches_oracle(bits):
    """The GPU exhaustive parity check's restatement (tests/_util.codes_f64 + quant_epilogue_ref: f64
    GEMM of the packed codes, the epilogue as torch IEEE ops) equals oracle_gg_quant bit for bit,
    including zero accumulators, extreme codes and scales that overflow fp16."""
    from tests._util import codes_f64, quant_epilogue_ref

    rng = np.random.default_rng(bits)
    M, N, K = 37, 45, 512
    qmax = (1 << (bits - 1)) - 1
    qa = rng.integers(-qmax, qmax + 1, (M, K)).astype(np.int8)
    qb = rng.integers(-qmax, qmax + 1, (N, K)).astype(np.int8)
    qa[0] = 0                     # zero accumulators (+0, never -0)
    qa[1], qb[1] = qmax, -qmax    # extreme sums
    A = pack_wxax(torch.from_numpy(qa), bits).view(torch.uint8).numpy()
    B = pack_wxax(torch.from_numpy(qb), bits).view(torch.uint8).numpy()
    sa = (rng.random(M) * 0.02 + 1e-4).astype(np.float16)
    sb = (rng.random(N) * 0.02 + 1e-4).astype(np.float16)
    sa[2], sb[3] = 60000.0, 60000.0  # fp16_rn(sa * sb) = inf on row 2 x column 3
    ref = oracle.gg_quant(A, B, sa, sb, M, N, K, bits)
    acc = codes_f64(torch.from_numpy(A), M, bits, K) @ codes_f64(torch.from_numpy(B), N, bits, K).T
    assert torch.equal(acc, torch.from_numpy(qa.astype(np.float64) @ qb.astype(np.float64).T))
    got = quant_epilogue_ref(acc, torch.from_numpy(sa), torch.from_numpy(sb)).numpy()
    g16, r16 = got.view(np.uint16), ref.view(np.uint16)
    both_nan = np.isnan(got) & np.isnan(ref)
    assert ((g16 == r16) | both_nan).all()
