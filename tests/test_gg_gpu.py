"""GPU parity tests: the HIP GroupGEMM (through the C-ABI) against the CPU oracle.

Bar: bit-exact for w8a8 / w4a4 (int path), fp16 within 1e-3 relative (+ cancellation floor).
Edge cases mirror what the reference kernels handle (tail M tiles: mm_tile.cuh:253, 617-641;
M = 0 problems; mixed qtypes in one fused launch: compose_kernel.py:150-224) plus N tails,
K tails inside a 128-byte stage and strided C (N-slices) that the reference does not support.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import FP16, W4A4, W8A8, GroupGemm, Problem, QParams, group_gemm, groupgemm_reference_abi
from tests._util import HostProblem, assert_f16_close, exact_compare

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _check(hps):
    for hp in hps:
        out, ref = hp.result(), hp.expected()
        if exact_compare(hp.q):  # int32 accumulation: bit-exact
            mism = np.count_nonzero(out.view(np.uint16) != ref.view(np.uint16))
            assert mism == 0, f"{hp.q.qcfg} M={hp.M} N={hp.N} K={hp.K}: {mism} mismatching outputs"
        else:
            assert_f16_close(out, ref, hp.K)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nat.lib()


PROD = nat.production_variants()  # every correct compiled variant (abl_* excluded)


def _kbytes_ok(variant, K, q):
    return True  # every variant handles K tails (multiples of 16 bytes)


@pytest.mark.parametrize("variant", PROD)
@pytest.mark.parametrize("q", [FP16, W8A8, W4A4], ids=["fp16", "w8a8", "w4a4"])
def test_single_qtype_edge_shapes(q, variant):
    shapes = [(1, 128, 256), (17, 256, 128), (130, 128, 384), (257, 136, 512), (64, 8, 1024), (300, 520, 512),
              (513, 264, 256)]
    shapes = [s for s in shapes if _kbytes_ok(variant, s[2], q)]
    hps = [HostProblem(M, N, K, q, seed=100 + i, device=DEV) for i, (M, N, K) in enumerate(shapes)]
    group_gemm([h.problem for h in hps], variant=variant)
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("variant", PROD)
def test_mixed_fused_launch(variant):
    specs = [(300, 256, 256, W8A8), (0, 256, 256, W4A4), (129, 384, 512, W4A4), (77, 128, 192, FP16),
             (513, 256, 128, W8A8), (5, 128, 64, W4A4), (256, 256, 256, FP16), (384, 512, 1024, W8A8)]
    specs = [s for s in specs if _kbytes_ok(variant, s[2], s[3])]
    hps = [HostProblem(M, N, K, q, seed=7 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)
    # relaunch on the same plan is idempotent
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("variant", PROD)
@pytest.mark.parametrize("q", [W8A8, W4A4, FP16], ids=["w8a8", "w4a4", "fp16"])
def test_k_tail_inside_stage(q, variant):
    # K bytes not a multiple of the 128-B stage: the tail must not change the sum
    bits = 16 if not q.is_quant else q.a_bits
    hps = [HostProblem(70 + 61 * t, 128 + 8 * t, (128 * 8 // bits) * 3 + (128 // bits) * t, q, seed=3 + t, device=DEV)
           for t in range(1, 8)]  # 3 full stages + 16..112 bytes
    group_gemm([h.problem for h in hps], variant=variant)
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("variant", PROD)
def test_strided_c_nslices(variant):
    # two N-slices of one logical problem written into one C buffer with ldc = N_total
    M, N, K = 200, 512, 256
    C = torch.full((M, N), float("nan"), dtype=torch.float16, device=DEV)
    h0 = HostProblem(M, 256, K, W8A8, seed=11, device=DEV, C=C, c_col0=0)
    h1 = HostProblem(M, 256, K, W8A8, seed=12, device=DEV, C=C, c_col0=256)
    group_gemm([h0.problem, h1.problem], variant=variant)
    torch.cuda.synchronize()
    full = C.cpu().numpy()
    assert (full[:, :256].view(np.uint16) == h0.expected().view(np.uint16)).all()
    assert (full[:, 256:].view(np.uint16) == h1.expected().view(np.uint16)).all()


def test_reference_abi_shim():
    specs = [(33, 128, 256, W8A8), (65, 256, 512, W4A4), (20, 128, 128, FP16)]
    hps = [HostProblem(M, N, K, q, seed=21 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]

    def ptrs(get):
        return torch.tensor([get(h.problem) for h in hps], dtype=torch.int64, device=DEV)

    groupgemm_reference_abi(
        ptrs(lambda p: p.A.data_ptr()), ptrs(lambda p: p.B.data_ptr()),
        ptrs(lambda p: 0 if p.scale_a is None else p.scale_a.data_ptr()),
        ptrs(lambda p: 0 if p.scale_b is None else p.scale_b.data_ptr()), ptrs(lambda p: p.C.data_ptr()),
        [(h.M, h.N, h.K) for h in hps], [h.q for h in hps])
    torch.cuda.synchronize()
    _check(hps)


def test_unsupported_qtype_raises():
    h = HostProblem(16, 128, 128, W8A8, seed=1, device=DEV)
    p = h.problem
    from mxmoe_amd.groupgemm import QParams
    p.q = QParams(4, 16, -1, False)  # w4a16 asym: not compiled (reference: "quant type not supported")
    with pytest.raises(nat.GGError, match="quant type not supported"):
        group_gemm([p])


@pytest.mark.parametrize("variant", PROD)
def test_graph_capture_replay(variant):
    hps = [HostProblem(150, 256, 512, W8A8, seed=31, device=DEV), HostProblem(90, 128, 256, W4A4, seed=32, device=DEV)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        gg.launch(s)
    for h in hps:
        h.problem.C.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    _check(hps)



def test_nslice_views_match_full_call():
    """dist.nslice_plan work lists run as strided problem views (B rows / C columns of the full
    problems) reproduce the full call bit-for-bit: the strong-scaling path's per-rank compute."""
    from mxmoe_amd.dist import nslice_plan
    from mxmoe_amd.harness import build_layer_inputs, slice_problem
    from mxmoe_amd.workload import QShape

    shapes = [QShape([300, 1024, 512], 8, 8), QShape([77, 512, 256], 4, 4), QShape([1000, 2048, 384]),
              QShape([0, 256, 256], 8, 8), QShape([513, 768, 1408], 4, 4)]
    full = build_layer_inputs(shapes, device=DEV, seed=3)
    group_gemm(full.problems)
    torch.cuda.synchronize()
    ref = [p.C.clone() for p in full.problems]
    for world in (2, 3):
        for p in full.problems:
            p.C.fill_(float("nan"))
        for work in nslice_plan(shapes, world, target_frac=0.3):
            probs = [slice_problem(full.problems[w.problem], w.n0, w.n1) for w in work]
            if probs:
                group_gemm(probs)
        torch.cuda.synchronize()
        for i, (p, r) in enumerate(zip(full.problems, ref)):
            if p.M:
                assert torch.equal(p.C.view(torch.int16), r.view(torch.int16)), (world, i)


B3 = [ln.split()[1] for ln in nat.list_variants()].index("v2x_256x256_w8_b3_buf_spread_edma")


@pytest.mark.parametrize("variant", [None, B3], ids=["auto", "v2x"])
@pytest.mark.parametrize("q", [FP16, W8A8, W4A4, QParams(16, 4, 128, False)], ids=["fp16", "w8a8", "w4a4", "w4a16g128"])
def test_splitk_long_k_low_fill(q, variant):
    """Low-fill calls with a long K (the shared expert's down at small batch) are split along K;
    the last slice reduces the partial slabs in slice order: int paths stay bit-exact, results
    are deterministic, and the arrival counters reset for the next launch. Also with the 3-stage
    B ring forced (its mainloop feeds the same split-K hand-off)."""
    specs = [(512, 2048, 5632), (40, 2048, 1408), (3, 256, 1408)]
    hps = [HostProblem(M, N, K, q, seed=90 + i, device=DEV) for i, (M, N, K) in enumerate(specs)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    assert gg.info.splitk_slabs > 0
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)
    first = [h.problem.C.clone() for h in hps]
    for _ in range(3):
        gg.launch()
    torch.cuda.synchronize()
    for h, c in zip(hps, first):
        assert torch.equal(h.problem.C.view(torch.int16), c.view(torch.int16))


@pytest.mark.parametrize("q,K", [(W8A8, 4224), (W4A4, 4224), (FP16, 1408), (QParams(16, 4, 128, False), 1408)],
                         ids=["w8a8", "w4a4", "fp16", "w4a16g128"])
def test_splitk_slices_on_different_xcds(q, K):
    """Split groups whose slices land on different XCDs (blockIdx % 8 differs, so different L2s):
    the partial slabs are written with L2-bypassing stores and the arrival counter is a device-scope
    atomic, so the last slice must still read every other slice's partials. The planner check in
    tests/test_planner.py pins that these shapes do scatter slices across XCDs."""
    from tests.test_planner import cross_xcd_split_groups

    hps = [HostProblem(128, 2048, K, q, seed=140, device=DEV), HostProblem(40, 256, 1408, q, seed=141, device=DEV)]
    gg = GroupGemm([h.problem for h in hps])
    tiles, _ = nat.plan_tiles([h.problem.to_c() for h in hps], gg.variant)
    assert cross_xcd_split_groups(tiles) > 0
    for _ in range(2):  # second launch: counters were reset by the first
        for h in hps:
            h.problem.C.fill_(float("nan"))
        gg.launch()
        torch.cuda.synchronize()
        _check(hps)


@pytest.mark.parametrize("q", [FP16, W8A8], ids=["fp16", "w8a8"])
def test_64bit_offsets_large_c(q):
    """C of 65536 x 33024 (2.16e9 elements > 2^31): row offsets into C (and A) need 64-bit address
    arithmetic in the DMA sources and the epilogue stores. Checked on the last rows and columns
    against a torch fp32 reference of the same op (fp16: within tolerance; w8a8: bit-exact, the
    reference epilogue fp16(f32(acc) * f32(fp16(sa * sb))) with |acc| < 2^24). The pack_wxax byte
    order is the same permutation on A and B, so raw int8 rows stand in for packed ones."""
    M, N, K = 65536, 33024, 128
    g = torch.Generator(device=DEV).manual_seed(5)
    if q.is_quant:
        A = torch.randint(-127, 128, (M, K), generator=g, device=DEV, dtype=torch.int8).view(torch.uint8)
        B = torch.randint(-127, 128, (N, K), generator=g, device=DEV, dtype=torch.int8).view(torch.uint8)
        sa = (torch.rand(M, generator=g, device=DEV) * 1e-3 + 1e-4).half()
        sb = (torch.rand(N, generator=g, device=DEV) * 1e-3 + 1e-4).half()
    else:
        A = (torch.rand(M, K, generator=g, device=DEV) * 2 - 1).half()
        B = (torch.rand(N, K, generator=g, device=DEV) * 2 - 1).half()
        sa = sb = None
    C = torch.empty(M, N, dtype=torch.float16, device=DEV)
    group_gemm([Problem(A=A, B=B, C=C, M=M, N=N, K=K, q=q, scale_a=sa, scale_b=sb)])
    torch.cuda.synchronize()
    rows = torch.tensor([0, 1, 32767, 32768, 50000, 65534, 65535], device=DEV)
    cols = torch.cat([torch.arange(0, 64, device=DEV), torch.arange(N - 64, N, device=DEV)])
    got = C[rows][:, cols].float()
    if q.is_quant:
        acc = A[rows].view(torch.int8).float() @ B[cols].view(torch.int8).float().t()  # exact: |acc| < 2^24
        s = (sa[rows][:, None] * sb[cols][None, :]).float()  # fp16 products, correctly rounded
        ref = (acc * s).half().float()
        assert torch.equal(got, ref)
    else:
        ref = A[rows].float() @ B[cols].float().t()
        assert torch.allclose(got, ref, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))
    del C
    torch.cuda.empty_cache()


def _shim_call(hps, pad_byte=0):
    def ptrs(get):
        return torch.tensor([get(h.problem) for h in hps], dtype=torch.int64, device=DEV)

    groupgemm_reference_abi(
        ptrs(lambda p: p.A.data_ptr()), ptrs(lambda p: p.B.data_ptr()),
        ptrs(lambda p: 0 if p.scale_a is None else p.scale_a.data_ptr()),
        ptrs(lambda p: 0 if p.scale_b is None else p.scale_b.data_ptr()), ptrs(lambda p: p.C.data_ptr()),
        [(h.M, h.N, h.K) for h in hps], [h.q for h in hps], pad_byte=pad_byte)


@pytest.mark.parametrize("pad_byte", [0x01, 0x02, 0xAB])
def test_reference_abi_shim_ignores_qparams_padding(pad_byte):
    """The reference's QParams constructors leave the 3 bytes after `sym` uninitialised
    (quantize.cuh:19-20): whatever they hold, the shim computes the default-format result."""
    specs = [(33, 128, 256, W8A8), (65, 256, 512, W4A4), (20, 128, 128, FP16)]
    hps = [HostProblem(M, N, K, q, seed=141 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    _shim_call(hps, pad_byte=pad_byte)
    torch.cuda.synchronize()
    _check(hps)


def test_reference_abi_shim_growing_problem_count_and_release():
    """The shim's cached per-device workspace grows between calls (P 2 -> 9, more tiles) and is
    released explicitly; every call's output is exact."""
    small = [HostProblem(33, 128, 256, W8A8, seed=61, device=DEV), HostProblem(17, 128, 128, FP16, seed=62, device=DEV)]
    _shim_call(small)
    torch.cuda.synchronize()
    _check(small)
    big = [HostProblem(300 + 40 * i, 512, 512, [W8A8, W4A4, FP16][i % 3], seed=70 + i, device=DEV) for i in range(9)]
    _shim_call(big)
    _shim_call(small)  # back to the small plan on the grown buffers
    torch.cuda.synchronize()
    _check(big)
    _check(small)
    nat.check(nat.lib().mxmoe_gg_release_shim_workspaces())
    _shim_call(small)  # re-allocates after a release
    torch.cuda.synchronize()
    _check(small)


def test_reference_abi_shim_rejects_null_scale():
    hps = [HostProblem(33, 128, 256, W8A8, seed=81, device=DEV)]
    hps[0].problem.scale_b = None  # the gathered pointer is NULL: an error code, not a GPU fault
    with pytest.raises(nat.GGError, match="NULL scale"):
        _shim_call(hps)


def test_reference_abi_shim_plan_cache():
    """Same shapes call after call reuse the cached plan: with the same buffers (nothing uploaded),
    with new buffers (pointer columns re-uploaded), and a NULL scale still fails on a cache hit."""
    specs = [(300, 256, 512, W8A8), (65, 256, 512, W4A4), (20, 128, 128, FP16), (0, 128, 128, W8A8)]
    a = [HostProblem(M, N, K, q, seed=90 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    b = [HostProblem(M, N, K, q, seed=190 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    _shim_call(a)  # plans and caches
    torch.cuda.synchronize()
    _check(a)
    for h in a:
        h.problem.C.fill_(float("nan"))
    _shim_call(a)  # cache hit, same pointers
    torch.cuda.synchronize()
    _check(a)
    _shim_call(b)  # cache hit, new pointers
    torch.cuda.synchronize()
    _check(b)
    for h in a:
        h.problem.C.fill_(float("nan"))
    _shim_call(a)  # and back
    torch.cuda.synchronize()
    _check(a)
    b[0].problem.scale_a = None
    with pytest.raises(nat.GGError, match="NULL scale"):
        _shim_call(b)


def test_rebind_all_empty_plan_rejects_non_empty_problems():
    """a plan whose problems are all empty has an empty table order; rebinding it with
    non-empty problems must fail the plan-signature check (not take the fast path and leave C
    unwritten). The same empty shapes rebind fine; forgetting the workspace keeps that true."""
    empty = [HostProblem(0, 128, 256, W8A8, seed=301, device=DEV), HostProblem(0, 256, 128, FP16, seed=302, device=DEV)]
    gg = GroupGemm([h.problem for h in empty])
    assert gg.total_tiles == 0
    gg.rebind([h.problem for h in empty])  # same (empty) shapes: accepted
    full = [HostProblem(64, 128, 256, W8A8, seed=303, device=DEV), HostProblem(32, 256, 128, FP16, seed=304, device=DEV)]
    with pytest.raises(nat.GGError, match="differ from the planned call"):
        gg.rebind([h.problem for h in full])
    nat.check(nat.lib().mxmoe_gg_forget_workspace(ctypes.c_void_p(gg.workspace.data_ptr())))
    gg.rebind([h.problem for h in empty])  # planner path after the key is dropped: still accepted
    with pytest.raises(nat.GGError, match="differ from the planned call"):
        gg.rebind([h.problem for h in full])
