"""w4a4_g128_sym: int4 A and B with one fp16 scale per 128-K group.

Reference: cta_gemm_w4a4g128 (mxmoe/kernels/src/include/cta_gemm.cuh:610-772) — per group an exact
int32 dot product, folded as out += f32(acc_g) * f32(fp16(sa_g * sb_g)) (one FFMA), C = fp16(out);
scales [K/128][M] / [K/128][N] (permute_scale, quantize.cuh:299-315; test.cu:240-313).

CPU tests pin the oracle (oracle/gg_oracle.c: oracle_gg_quant_grouped) and the host quantiser to the
golden vectors make_golden.py produced with the reference's quant_minmax(t, 4, 128, True); GPU tests
hold the HIP kernel (gg_tile_g128) to the oracle bit for bit.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import FP16, W4A4, W4A4_G128, W8A8, GroupGemm, Problem, QParams, group_gemm
from mxmoe_amd.quantize import quant_rtn_sym
from oracle import oracle
from tests._util import HostProblem, assert_f16_close

GOLD = Path(__file__).resolve().parent / "golden"
DEV = "cuda"


def _golden():
    d = np.load(GOLD / "gg_w4a4g128_small.npz")
    for i in range(int(d["P"])):
        M, N, K = (int(x) for x in d[f"p{i}_shape"])
        yield i, M, N, K, d


# ------------------------------------------------------------------------------------------ CPU

def test_group_quant_matches_reference_quant_minmax():
    d = np.load(GOLD / "quant_g128_golden.npz")
    x, q_ref, s_ref = d["x_4"], d["q_4"], d["scale_4"]
    rows, K = x.shape
    s_perm = np.ascontiguousarray(s_ref.reshape(rows, K // 128).T).reshape(-1)  # permute_scale
    q_o, s_o = oracle.quant_rtn_sym_grouped(x, 4, 128)
    assert (q_o == q_ref).all()
    assert (s_o.view(np.uint16) == s_perm.view(np.uint16)).all()
    q_t, s_t = quant_rtn_sym(torch.from_numpy(x), 4, 128)
    assert (q_t.numpy() == q_ref).all()
    assert (s_t.numpy().view(np.uint16) == s_perm.view(np.uint16)).all()


def test_oracle_grouped_bit_exact_vs_golden():
    for i, M, N, K, d in _golden():
        C = oracle.gg_quant_grouped(d[f"p{i}_A"], d[f"p{i}_B"], d[f"p{i}_sa"], d[f"p{i}_sb"], M, N, K, 4, 128)
        assert (C.view(np.uint16) == d[f"p{i}_C"].view(np.uint16)).all(), f"problem {i}"
        assert (oracle.unpack_wxax(d[f"p{i}_A"], 4, K) == d[f"p{i}_qa"]).all()


def test_grouped_with_one_group_equals_per_channel():
    # K = 128: one group, so the fold is fma(acc, s, 0) = the per-channel epilogue 0 + acc * s
    rng = np.random.default_rng(3)
    M, N, K = 9, 16, 128
    A = rng.integers(0, 256, (M, K // 2), dtype=np.uint8)
    B = rng.integers(0, 256, (N, K // 2), dtype=np.uint8)
    sa = (rng.random(M) * 0.1).astype(np.float16)
    sb = (rng.random(N) * 0.1).astype(np.float16)
    c1 = oracle.gg_quant_grouped(A, B, sa, sb, M, N, K, 4, 128)
    c2 = oracle.gg_quant(A, B, sa, sb, M, N, K, 4)
    assert (c1.view(np.uint16) == c2.view(np.uint16)).all()


def _ws(probs, variant=nat.VARIANT_AUTO):
    arr = (nat.GGProblemC * len(probs))(*[p.to_c() for p in probs])
    return nat.workspace_size(arr, len(probs), variant)


def _meta_problem(M, N, K, q):
    t = torch.empty(0)
    return Problem(A=t, B=t, C=t, M=M, N=N, K=K, q=q)


def test_planner_accepts_g128_and_rejects_bad_shapes():
    assert _ws([_meta_problem(300, 256, 1408, W4A4_G128), _meta_problem(20, 256, 2048, W8A8)]) > 0
    with pytest.raises(nat.GGError, match="K % 128"):
        _ws([_meta_problem(64, 256, 192, W4A4_G128)])
    with pytest.raises(nat.GGError, match="not supported"):
        _ws([_meta_problem(64, 256, 256, QParams(4, 4, 64, True))])
    v3 = next(int(ln.split()[0]) for ln in nat.list_variants() if ln.split()[1].startswith("v3"))
    with pytest.raises(nat.GGError, match="not supported"):  # the v3 kernels have no g128 body
        _ws([_meta_problem(64, 256, 256, W4A4_G128)], v3)


def test_variant_listing_names_g128():
    lines = [ln for ln in nat.list_variants() if ln.split()[1].startswith("v2x")]
    assert any("w4a4_g128_sym=TileConfig(BM=256, BN=256, BK=256" in ln for ln in lines)


# ------------------------------------------------------------------------------------------ GPU

V2 = [int(ln.split()[0]) for ln in nat.list_variants() if ln.split()[1].startswith("v2")]


def _check(hps):
    for hp in hps:
        out, ref = hp.result(), hp.expected()
        if hp.q.is_quant and not hp.q.is_weight_only:
            mism = np.count_nonzero(out.view(np.uint16) != ref.view(np.uint16))
            assert mism == 0, f"{hp.q.qcfg} M={hp.M} N={hp.N} K={hp.K}: {mism} mismatching outputs"
        else:
            assert_f16_close(out, ref, hp.K)


@pytest.fixture()
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nat.lib()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [nat.VARIANT_AUTO] + V2)
def test_g128_golden_vectors(gpu, variant):
    probs, exp = [], []
    for i, M, N, K, d in _golden():
        C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=DEV)
        probs.append(Problem(A=torch.from_numpy(d[f"p{i}_A"]).to(DEV), B=torch.from_numpy(d[f"p{i}_B"]).to(DEV), C=C,
                             M=M, N=N, K=K, q=W4A4_G128, scale_a=torch.from_numpy(d[f"p{i}_sa"]).to(DEV),
                             scale_b=torch.from_numpy(d[f"p{i}_sb"]).to(DEV)))
        exp.append(d[f"p{i}_C"])
    group_gemm(probs, variant=None if variant == nat.VARIANT_AUTO else variant)
    torch.cuda.synchronize()
    for p, ref in zip(probs, exp):
        out = p.C[: p.M, : p.N].cpu().numpy()
        assert (out.view(np.uint16) == ref.view(np.uint16)).all(), f"M={p.M} N={p.N} K={p.K}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", V2)
def test_g128_edge_shapes(gpu, variant):
    # M tails (1, 17, 127, 129, 257), N tails (8, 136, 264), K = 1 .. 16 groups incl. odd group counts
    # (the second group of the last 256-element stage missing), K = 5632 (shared-expert down)
    shapes = [(1, 128, 128), (17, 256, 384), (127, 136, 1408), (129, 8, 256), (257, 264, 2048), (64, 256, 5632),
              (300, 520, 640)]
    hps = [HostProblem(M, N, K, W4A4_G128, seed=200 + i, device=DEV) for i, (M, N, K) in enumerate(shapes)]
    group_gemm([h.problem for h in hps], variant=variant)
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.gpu
def test_g128_mixed_with_every_qtype(gpu):
    specs = [(300, 256, 1408, W4A4_G128), (129, 384, 512, W4A4), (77, 128, 192, FP16), (0, 256, 256, W4A4_G128),
             (513, 256, 2048, W8A8), (260, 256, 1408, QParams(16, 4, 128, False)), (33, 128, 128, W4A4_G128)]
    hps = [HostProblem(M, N, K, q, seed=300 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    gg = GroupGemm([h.problem for h in hps])
    assert gg.info.qtype_mask & (1 << 5)
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.gpu
def test_g128_strided_c_and_relaunch_deterministic(gpu):
    C = torch.full((200, 640), float("nan"), dtype=torch.float16, device=DEV)
    hps = [HostProblem(200, 256, 1024, W4A4_G128, seed=41, device=DEV, C=C, c_col0=0),
           HostProblem(200, 384, 1024, W4A4_G128, seed=42, device=DEV, C=C, c_col0=256)]
    gg = GroupGemm([h.problem for h in hps])
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)
    first = C.clone()
    gg.launch()
    torch.cuda.synchronize()
    assert torch.equal(first.view(torch.int16), C.view(torch.int16))


@pytest.mark.gpu
def test_g128_full_size_layer11_sampled(gpu):
    """qwen2_moe layer-11 bs=8192 with every problem w4a4_g128: a random 48 x 48 sample of each
    problem's outputs against the oracle (C[rows, cols] depends only on A[rows], B[cols], and the
    group scales of those rows / columns)."""
    from mxmoe_amd.harness import build_layer_inputs
    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    wl = load_workload(qwen2_layer11_workload(8192, qstr="w4a4_g128_sym"))["layer-11"]
    rng = np.random.default_rng(5)
    for gg in ("gate_up", "down"):
        inp = build_layer_inputs(wl[gg])
        GroupGemm(inp.problems).launch()
        torch.cuda.synchronize()
        for p in inp.problems:
            G = p.K // 128
            rows = np.sort(rng.choice(p.M, size=min(48, p.M), replace=False))
            cols = np.sort(rng.choice(p.N, size=min(48, p.N), replace=False))
            rt, ct = torch.from_numpy(rows).to(DEV), torch.from_numpy(cols).to(DEV)
            A = p.A.index_select(0, rt).cpu().numpy()
            B = p.B.index_select(0, ct).cpu().numpy()
            sa = p.scale_a.view(G, p.M).index_select(1, rt).contiguous().cpu().numpy().reshape(-1)
            sb = p.scale_b.view(G, p.N).index_select(1, ct).contiguous().cpu().numpy().reshape(-1)
            ref = oracle.gg_quant_grouped(A, B, sa, sb, len(rows), len(cols), p.K, 4, 128)
            out = p.C.index_select(0, rt).index_select(1, ct).cpu().numpy()
            assert (out.view(np.uint16) == ref.view(np.uint16)).all(), f"{gg} M={p.M} N={p.N} K={p.K}"
        del inp
        torch.cuda.empty_cache()
