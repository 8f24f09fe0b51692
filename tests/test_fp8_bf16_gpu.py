"""GPU parity of the w8a8_g-1_sym_E4M3 (OCP fp8, block-scaled K=128 MFMA with unit scales) and bf16
tile bodies against the CPU oracle (oracle_gg_e4m3 / oracle_gg_bf16), through the C-ABI.

Bar: fp16 tolerance (1e-3 relative + cancellation floor, tests/_util.py) — both accumulate in f32
in an unspecified order — and BIT-EXACT on the small-integer known-answer test, where every partial
sum is an integer below 2^24 (so any summation order gives the same f32), which pins the fp8
fragment layout and the epilogue exactly.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import BF16, FP16, W4A4, W8A8, W8A8_E4M3, GroupGemm, Problem, group_gemm, groupgemm_reference_abi
from mxmoe_amd.quantize import pack_e4m3
from oracle import oracle
from tests._util import HostProblem, assert_f16_close, exact_compare

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nat.lib()


def _variants(qcfg):
    return nat.production_variants(qcfg)


def _check(hps):
    for hp in hps:
        out, ref = hp.result(), hp.expected()
        if exact_compare(hp.q):
            assert (out.view(np.uint16) == ref.view(np.uint16)).all(), f"{hp.q.qcfg} M={hp.M} N={hp.N} K={hp.K}"
        else:
            assert_f16_close(out, ref, hp.K)


SHAPES = [(1, 128, 256), (17, 256, 128), (130, 128, 384), (257, 136, 512), (64, 8, 1024), (300, 520, 512),
          (513, 264, 256), (70, 256, 2048)]


@pytest.mark.parametrize("q", [W8A8_E4M3, BF16], ids=["e4m3", "bf16"])
def test_edge_shapes_every_variant(q):
    vs = _variants(q.qcfg)
    assert vs, f"no variant implements {q.qcfg}"
    for v in vs:
        hps = [HostProblem(M, N, K, q, seed=200 + i, device=DEV) for i, (M, N, K) in enumerate(SHAPES)]
        group_gemm([h.problem for h in hps], variant=v)
        torch.cuda.synchronize()
        _check(hps)


@pytest.mark.parametrize("q", [W8A8_E4M3, BF16], ids=["e4m3", "bf16"])
def test_k_tail_inside_stage(q):
    per_byte = 1 if q.is_fp8 else 2  # bytes per element
    for v in _variants(q.qcfg):
        hps = [HostProblem(70 + 61 * t, 128 + 8 * t, (384 + 16 * t) // per_byte, q, seed=30 + t, device=DEV)
               for t in range(1, 8)]  # 3 full 128-B stages + 16..112 bytes
        group_gemm([h.problem for h in hps], variant=v)
        torch.cuda.synchronize()
        _check(hps)


def test_e4m3_small_integer_known_answer_bit_exact():
    """Integers in [-8, 8] are exact e4m3 values; with K = 2048 every partial sum is an integer
    < 2^24, exact in f32 in any order, so the GPU must equal the oracle bit for bit."""
    g = torch.Generator().manual_seed(9)
    M, N, K = 300, 264, 2048
    ia = torch.randint(-8, 9, (M, K), generator=g).float()
    ib = torch.randint(-8, 9, (N, K), generator=g).float()
    qa = ia.to(torch.float8_e4m3fn).view(torch.uint8)
    qb = ib.to(torch.float8_e4m3fn).view(torch.uint8)
    sa = (torch.rand(M, generator=g) * 0.01 + 0.001).half()
    sb = (torch.rand(N, generator=g) * 0.01 + 0.001).half()
    A, B = pack_e4m3(qa), pack_e4m3(qb)
    ref = oracle.gg_e4m3(A.numpy(), B.numpy(), sa.numpy(), sb.numpy(), M, N, K)
    # the exact integer sums, independently
    acc = (ia.double() @ ib.double().T).float()
    s16 = (sa.float()[:, None] * sb.float()[None, :]).half().float()
    assert (ref.view(np.uint16) == (0.0 + acc * s16).half().numpy().view(np.uint16)).all()
    for v in _variants("w8a8_g-1_sym_E4M3"):
        C = torch.full((M, N), float("nan"), dtype=torch.float16, device=DEV)
        group_gemm([Problem(A=A.to(DEV), B=B.to(DEV), C=C, M=M, N=N, K=K, q=W8A8_E4M3, scale_a=sa.to(DEV),
                            scale_b=sb.to(DEV))], variant=v)
        torch.cuda.synchronize()
        out = C.cpu().numpy()
        assert (out.view(np.uint16) == ref.view(np.uint16)).all(), f"variant {v}: {(out != ref).sum()} differ"


def test_mixed_launch_every_type():
    """fp8 + bf16 with the other types in one fused launch (the every-body fallback kernel)."""
    specs = [(300, 256, 256, W8A8_E4M3), (129, 384, 512, W4A4), (77, 128, 192, FP16), (200, 256, 384, BF16),
             (0, 256, 256, W8A8_E4M3), (513, 256, 128, W8A8), (33, 136, 2048, W8A8_E4M3), (5, 128, 64, BF16)]
    for v in _variants("w8a8_g-1_sym_E4M3"):
        hps = [HostProblem(M, N, K, q, seed=70 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
        gg = GroupGemm([h.problem for h in hps], variant=v)
        gg.launch()
        torch.cuda.synchronize()
        _check(hps)


@pytest.mark.parametrize("q", [W8A8_E4M3, BF16], ids=["e4m3", "bf16"])
def test_low_fill_split_k(q):
    """One long-K tile: the planner splits it along K (slabs summed in slice order)."""
    K = 8192 if q.is_fp8 else 4096
    for v in _variants(q.qcfg):
        hps = [HostProblem(256, 256, K, q, seed=5, device=DEV), HostProblem(96, 256, K, q, seed=6, device=DEV)]
        gg = GroupGemm([h.problem for h in hps], variant=v)
        assert gg.info.splitk_slabs > 0
        gg.launch()
        torch.cuda.synchronize()
        _check(hps)


def test_reference_abi_shim_carries_fmt():
    specs = [(33, 128, 256, W8A8_E4M3), (65, 256, 512, BF16), (20, 128, 128, W8A8)]
    hps = [HostProblem(M, N, K, q, seed=41 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]

    def ptrs(get):
        return torch.tensor([get(h.problem) for h in hps], dtype=torch.int64, device=DEV)

    groupgemm_reference_abi(
        ptrs(lambda p: p.A.data_ptr()), ptrs(lambda p: p.B.data_ptr()),
        ptrs(lambda p: 0 if p.scale_a is None else p.scale_a.data_ptr()),
        ptrs(lambda p: 0 if p.scale_b is None else p.scale_b.data_ptr()), ptrs(lambda p: p.C.data_ptr()),
        [(h.M, h.N, h.K) for h in hps], [h.q for h in hps])
    torch.cuda.synchronize()
    _check(hps)
