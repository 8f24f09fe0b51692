"""CPU tests of the w8a8_g-1_sym_E4M3 and bf16 strategies (reference SUPPORTED_QCFG,
tile_config.py:40-106; QCFG_W8A8_E4M3 :192; MMA wrappers cuda_utils.cuh:385-410).

Parity pinning: the reference ships no E4M3 quantiser and no codegen branch for E4M3 / bf16
(compose_kernel.py:47-57), so there is no reference-produced output to pin against ("parity
unpinned" by the reference). What IS pinned here: the e4m3 code <-> value map and the
f32 -> e4m3 rounding of the C oracle against torch.float8_e4m3fn (an independent OCP implementation),
the product quantiser against the C oracle bit for bit, the 8-bit pack_wxax byte order, and the
oracle GroupGEMMs against plain f64 numpy.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import BF16, FP16, W8A8, W8A8_E4M3, QParams
from mxmoe_amd.quantize import pack_e4m3, pack_wxax, quant_e4m3, unpack_wxax
from mxmoe_amd.tile_config import MI355X_QCFG, SUPPORTED_QCFG, get_info_from_qcfg_str, variant_key
from mxmoe_amd.workload import QShape, parse_qstr
from oracle import oracle


def test_e4m3_decode_matches_torch_for_every_code():
    codes = np.arange(256, dtype=np.uint8)
    ours = oracle.e4m3_to_f32(codes)
    ref = torch.from_numpy(codes).view(torch.float8_e4m3fn).float().numpy()
    nan = np.isnan(ref)
    assert (np.isnan(ours) == nan).all()
    assert (ours[~nan].view(np.uint32) == ref[~nan].view(np.uint32)).all()  # incl. -0
    assert ours[0x7e] == 448.0 and ours[0x01] == 2.0 ** -9


def test_f32_to_e4m3_rounding_matches_torch():
    g = torch.Generator().manual_seed(0)
    vals = [torch.randn(4000, generator=g) * s for s in (1e-3, 0.05, 1.0, 30.0, 300.0)]
    finite = torch.from_numpy(np.arange(256, dtype=np.uint8)).view(torch.float8_e4m3fn).float()
    finite = finite[torch.isfinite(finite)]
    mids = (finite.sort().values[1:] + finite.sort().values[:-1]) / 2  # exact ties: round-half-even
    x = torch.cat(vals + [finite, mids, torch.tensor([447.9, 448.0, -448.0, 0.0, -0.0, 1e-9])]).clamp(-448, 448)
    ours = oracle.f32_to_e4m3(x.numpy())
    ref = x.to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    assert (ours == ref).all(), np.flatnonzero(ours != ref)[:10]


def test_product_quantiser_matches_oracle_bit_exact():
    g = torch.Generator().manual_seed(5)
    x = ((torch.rand(37, 272, generator=g) * 2 - 1) * torch.logspace(-4, 2, 37)[:, None]).half()
    x[3] = 0  # all-zero row: scale 1
    x[5, 7] = 60000.0  # large outlier row
    x[9] = 0
    x[9, 4], x[9, 100] = 1e-5, -3e-6  # tiny row: amax / 448 underflows fp16 -> scale 2^-14, codes kept
    q, s = quant_e4m3(x)
    qo, so = oracle.quant_e4m3(x.numpy())
    assert (s.numpy().view(np.uint16) == so.view(np.uint16)).all()
    assert (q.numpy() == qo).all()
    assert float(s[3]) == 1.0
    assert float(s[9]) == 2.0 ** -14 and (q[9].numpy() != 0).sum() == 2
    assert (s.float() >= 2.0 ** -14).all()


def test_pack_e4m3_is_pack_wxax_byte_order():
    g = torch.Generator().manual_seed(1)
    codes = torch.randint(0, 256, (9, 64), generator=g, dtype=torch.int32).to(torch.uint8)
    packed = pack_e4m3(codes)
    assert (packed.numpy() == oracle.pack_wxax(codes.view(torch.int8).numpy(), 8)).all()
    assert (unpack_wxax(packed, 8, 64).view(torch.uint8) == codes).all()
    assert (packed[:, 0] == codes[:, 1]).all() and (packed[:, 1] == codes[:, 0]).all()


def test_oracle_gg_e4m3_matches_f64_numpy():
    g = torch.Generator().manual_seed(2)
    M, N, K = 19, 24, 160
    a = (torch.rand(M, K, generator=g) * 2 - 1).half()
    b = (torch.rand(N, K, generator=g) * 2 - 1).half()
    qa, sa = quant_e4m3(a)
    qb, sb = quant_e4m3(b)
    C = oracle.gg_e4m3(pack_e4m3(qa).numpy(), pack_e4m3(qb).numpy(), sa.numpy(), sb.numpy(), M, N, K)
    acc = (oracle.e4m3_to_f32(qa.numpy()).astype(np.float64) @ oracle.e4m3_to_f32(qb.numpy()).astype(np.float64).T)
    s16 = (sa.numpy().astype(np.float32)[:, None] * sb.numpy().astype(np.float32)[None, :]).astype(np.float16)
    ref = (np.float32(0) + acc.astype(np.float32) * s16.astype(np.float32)).astype(np.float16)
    assert (C.view(np.uint16) == ref.view(np.uint16)).all()
    # and the quantised product is a faithful approximation of the fp16 GEMM
    exact = a.double().numpy() @ b.double().numpy().T
    assert np.linalg.norm(C.astype(np.float64) - exact) < 0.05 * np.linalg.norm(exact)


def test_oracle_gg_bf16_matches_f64_numpy():
    g = torch.Generator().manual_seed(3)
    M, N, K = 13, 40, 96
    a = (torch.rand(M, K, generator=g) * 2 - 1).bfloat16()
    b = (torch.rand(N, K, generator=g) * 2 - 1).bfloat16()
    C = oracle.gg_bf16(a.view(torch.int16).numpy().view(np.uint16), b.view(torch.int16).numpy().view(np.uint16), M, N, K)
    ref = (a.double() @ b.double().T).float().half().numpy()
    assert (C.view(np.uint16) == ref.view(np.uint16)).all()


def test_qcfg_names_round_trip():
    for q in MI355X_QCFG:
        p = QParams.from_qcfg(q)
        base = q.replace("_accfp16", "")
        assert p.qcfg == base, (q, p)
        assert get_info_from_qcfg_str(q)[:2] == (p.w_bits, p.a_bits)
    assert QParams.from_qcfg("w8a8_g-1_sym_E4M3") == W8A8_E4M3 and W8A8_E4M3.fmt_code == nat.FMT_E4M3
    assert QParams.from_qcfg("bf16") == BF16 and BF16.fmt_code == nat.FMT_BF16
    assert QParams.from_qcfg("fp16_accfp16") == FP16
    assert W8A8.fmt_code == nat.FMT_DEFAULT
    with pytest.raises(ValueError):
        QParams.from_qcfg("w4a16_g128_asym_bf16")  # weight-only with bf16 activations: not built
    assert set(MI355X_QCFG) <= set(SUPPORTED_QCFG)
    assert variant_key("fp16_accfp16") == "fp16" and variant_key("w4a16_g-1_sym_accfp16") == "w4a16"
    assert variant_key("w8a8_g-1_sym_E4M3") == "w8a8_g-1_sym_E4M3"


def test_workload_fmt_round_trip_keeps_reference_json():
    assert parse_qstr("w8a8_g-1_sym_E4M3") == {"w_bits": 8, "a_bits": 8, "gsize": -1, "sym": True, "fmt": "E4M3"}
    assert parse_qstr("bf16")["fmt"] == "bf16" and "fmt" not in parse_qstr("fp16_accfp16")
    assert "fmt" not in parse_qstr("w8a8_g-1_sym")  # reference qstrs give the reference dict
    s = QShape(shape=[5, 256, 128], w_bits=8, a_bits=8, fmt="E4M3")
    assert QShape.from_json(s.to_json()) == s and s.qcfg == "w8a8_g-1_sym_E4M3"
    assert "fmt" not in QShape(shape=[5, 256, 128], w_bits=8, a_bits=8).to_json()
    assert QShape(shape=[1, 8, 16], fmt="bf16").qcfg == "bf16"


def test_abi_qparams_padding_and_fmt_field():
    assert nat.MxmoeQParams.sym.offset == 12 and nat.MxmoeQParams.pad_.offset == 13
    assert ctypes.sizeof(nat.MxmoeQParams) == 16
    assert nat.GGProblemC.fmt.offset == nat.GGProblemC.sym.offset + 4
    assert nat.lib().mxmoe_gg_abi_version() == nat.ABI_VERSION


def _plan_error(probs, variant):
    P = len(probs)
    arr = (nat.GGProblemC * P)(*probs)
    n = ctypes.c_size_t()
    return nat.lib().mxmoe_gg_workspace_size(arr, P, variant, ctypes.byref(n))


def _prob(M, N, K, a, w, fmt, g=-1, sym=1):
    return nat.GGProblemC(A=0, B=0, scale_a=0, scale_b=0, C=0, M=M, N=N, K=K, a_bits=a, w_bits=w, gsize=g, sym=sym,
                          fmt=fmt, lda=0, ldb=0, ldc=0)


def test_host_planner_accepts_fp8_bf16_on_v2_only():
    v2 = nat.default_variant()
    assert _plan_error([_prob(300, 512, 2048, 8, 8, nat.FMT_E4M3), _prob(40, 256, 512, 16, 16, nat.FMT_BF16)], v2) == 0
    assert _plan_error([_prob(300, 512, 2048, 8, 8, nat.FMT_E4M3)], 0) == nat.MXMOE_GG_ERR_UNSUPPORTED  # v0
    assert _plan_error([_prob(300, 512, 2048, 4, 4, nat.FMT_E4M3)], v2) == nat.MXMOE_GG_ERR_UNSUPPORTED
    assert _plan_error([_prob(300, 512, 2048, 8, 8, nat.FMT_BF16)], v2) == nat.MXMOE_GG_ERR_UNSUPPORTED
    assert _plan_error([_prob(300, 512, 2048, 8, 8, 7)], v2) == nat.MXMOE_GG_ERR_UNSUPPORTED
    # AUTO resolves to a v2 variant that implements both
    arr = (nat.GGProblemC * 2)(_prob(300, 512, 2048, 8, 8, nat.FMT_E4M3), _prob(40, 256, 512, 16, 16, nat.FMT_BF16))
    v = nat.resolve_variant(arr, 2)
    assert nat.variant_supports(v, "w8a8_g-1_sym_E4M3") and nat.variant_supports(v, "bf16")
