"""Weight-only WxA16 GroupGEMM on the GPU vs the oracle (fp16 tolerance of tests/_util.py)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import FP16, W4A4, W8A8, GroupGemm, QParams, group_gemm
from tests._util import HostProblem, assert_f16_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
V2 = [int(ln.split()[0]) for ln in nat.list_variants() if ln.split()[1].startswith("v2")]
# weight-only-only kernels (wo3: 64-row tiles, 3 workgroups per CU)
WO = [v for v in nat.production_variants("w4a16_g-1_asym") if not nat.variant_supports(v, "w4a4_g128_sym")]
QS = [QParams(16, b, g, s) for b in (2, 4, 8) for g in (-1, 128) for s in (True, False)]


def _check(hps):
    for hp in hps:
        if hp.M:
            assert_f16_close(hp.result(), hp.expected(), hp.K)


@pytest.mark.parametrize("variant", V2 + WO)
@pytest.mark.parametrize("q", QS, ids=[q.qcfg for q in QS])
def test_weightonly_edge_shapes(q, variant):
    shapes = [(1, 128, 256), (17, 256, 128 if q.gsize == -1 else 256), (130, 136, 384), (257, 264, 512),
              (513, 512, 1408 if q.gsize == -1 else 1408), (0, 256, 256), (64, 8, 1024)]
    hps = [HostProblem(M, N, K, q, seed=300 + i, device=DEV) for i, (M, N, K) in enumerate(shapes)]
    group_gemm([h.problem for h in hps], variant=variant)
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("bits", [2, 4, 8])
def test_reference_format_weights_through_repack(bits):
    """B built in the reference's packed format (permute_weight + pack_weightonly), converted by
    mxmoe_gg_repack_weightonly, then run — the drop-in route for reference-packed weights."""
    hps = [HostProblem(M, N, K, QParams(16, bits, 128, False), seed=40 + i, device=DEV, ref_format=True)
           for i, (M, N, K) in enumerate([(300, 256, 1408), (77, 512, 2048)])]
    group_gemm([h.problem for h in hps])
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("variant", V2)
def test_all_quant_types_in_one_launch(variant):
    specs = [(300, 256, 256, W8A8), (129, 384, 512, W4A4), (77, 128, 192, FP16), (260, 256, 1408, QParams(16, 4, 128, False)),
             (33, 512, 2048, QParams(16, 8, -1, True)), (0, 256, 256, QParams(16, 4, -1, True)),
             (513, 264, 640, QParams(16, 4, 64, True)), (96, 256, 512, QParams(16, 2, 128, False))]
    hps = [HostProblem(M, N, K, q, seed=70 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    assert gg.info.qtype_mask == 0b1011111
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)


@pytest.mark.parametrize("variant", WO)
def test_wo3_weightonly_mix_and_split_k(variant):
    """Every weight-only width in one wo3 launch (the QM = 88 specialisation), plus a low-fill call
    whose long-K problem the planner splits along K (slab reduce in the 3-WG/CU kernel)."""
    assert WO, "no weight-only-only variant compiled"
    specs = [(260, 256, 1408, QParams(16, 4, 128, False)), (33, 512, 2048, QParams(16, 8, -1, True)),
             (0, 256, 256, QParams(16, 4, -1, True)), (513, 264, 640, QParams(16, 4, 64, True)),
             (96, 256, 512, QParams(16, 2, 128, False)), (7, 136, 1024, QParams(16, 8, 128, False))]
    hps = [HostProblem(M, N, K, q, seed=90 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    assert gg.info.lds_bytes == 78 * 1024  # 8-bit weight-only problems: the 2-WG/CU build
    gg.launch()
    torch.cuda.synchronize()
    _check(hps)
    # low fill: one 128 x 2048 x 5632 problem (the bs=128 shared-expert down shape) + 4 small ones
    hps = [HostProblem(128, 2048, 5632, QParams(16, 4, 128, False), seed=95, device=DEV)] + \
          [HostProblem(9, 2048, 1408, QParams(16, 4, 128, False), seed=96 + i, device=DEV) for i in range(4)]
    gg = GroupGemm([h.problem for h in hps], variant=variant)
    assert gg.info.splitk_slabs > 0, "expected a split-K plan"
    assert gg.info.lds_bytes == 52 * 1024  # 4-bit only: the 3-WG/CU build
    for _ in range(2):  # counters re-armed between launches
        gg.launch()
        torch.cuda.synchronize()
        _check(hps)


@pytest.mark.parametrize("variant", WO)
def test_wo3_w8a8_beside_weightonly_bit_exact(variant):
    """wo3's int8 body (64 x 128 tiles, plain v2 mainloop) beside weight-only problems: w8a8 edge
    shapes (M 1 / 17 / 130, N tails, K tails inside a 128-B stage, long K) bit-exact against the
    oracle in one launch with w4a16 problems; then the same with split-K (low fill, long K)."""
    specs = [(1, 128, 256, W8A8), (17, 136, 128, W8A8), (130, 264, 384 + 48, W8A8), (300, 520, 512, W8A8),
             (64, 8, 1024 + 16, W8A8), (77, 256, 1408, QParams(16, 4, -1, False)), (34, 2816, 2048, W8A8)]
    hps = [HostProblem(M, N, K, q, seed=110 + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
    for _ in range(2):
        GroupGemm([h.problem for h in hps], variant=variant).launch()
        torch.cuda.synchronize()
        for h in hps:
            if h.q.is_weight_only:
                assert_f16_close(h.result(), h.expected(), h.K)
            else:
                assert (h.result().view(np.uint16) == h.expected().view(np.uint16)).all(), (h.M, h.N, h.K)
        hps = [HostProblem(40, 1024, 8192, W8A8, seed=120, device=DEV),
               HostProblem(20, 512, 1024, QParams(16, 4, 128, False), seed=121, device=DEV)]


@pytest.mark.parametrize("variant", WO)
def test_wo3_fp16_and_w8a8_calls(variant):
    """wo3's fp16 and int8 bodies (64 x 128 tiles) on their own (QM = 1 / 2 builds, 3 WG/CU) and
    mixed with weight-only problems (the QM = 91 2-WG/CU build): edge shapes, K tails, a long-K
    low-fill split-K call; fp16 within the fp16 tolerance, w8a8 bit-exact."""
    edge = [(1, 128, 256), (17, 136, 128), (130, 264, 432), (300, 520, 512), (64, 8, 1040), (34, 2816, 2048)]
    sets = [[(M, N, K, FP16) for M, N, K in edge], [(M, N, K, W8A8) for M, N, K in edge],
            [(M, N, K, q) for (M, N, K), q in zip(edge, [FP16, W8A8, FP16, QParams(16, 4, -1, False), W8A8,
                                                           QParams(16, 8, 128, True)])],
            [(128, 2048, 5632, FP16), (9, 2048, 1408, FP16), (128, 2048, 5632, W8A8)]]
    for k, specs in enumerate(sets):
        hps = [HostProblem(M, N, K, q, seed=130 + 10 * k + i, device=DEV) for i, (M, N, K, q) in enumerate(specs)]
        gg = GroupGemm([h.problem for h in hps], variant=variant)
        for _ in range(2):
            gg.launch()
            torch.cuda.synchronize()
            for h in hps:
                if h.q.is_quant and not h.q.is_weight_only:
                    assert (h.result().view(np.uint16) == h.expected().view(np.uint16)).all(), (k, h.M, h.N, h.K)
                else:
                    assert_f16_close(h.result(), h.expected(), h.K)


@pytest.mark.parametrize("variant", [None] + WO)  # None: AUTO (wo3 at these batches)
@pytest.mark.parametrize("bs", [512, 128])
def test_w4a16_w8a8_layer_bs512_matches_oracle(bs, variant):
    """BASELINE's small-batch mixed scheme (bench config w4a16_w8a8_bs512): the qwen2_moe layer-11
    gate_up and down calls at bs = 512 with 1/16 of the blocks w8a8 and the rest w4a16_g-1_asym, ONE
    fused AUTO launch each; every problem against the oracle on a row / column sample (w8a8 bit-exact,
    w4a16 within the fp16 tolerance)."""
    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload, w4a16_w8a8_qconfig

    layer = load_workload(qwen2_layer11_workload(bs, qconfig=w4a16_w8a8_qconfig()))["layer-11"]
    rng = np.random.default_rng(bs)
    for gg in ("gate_up", "down"):
        shapes = layer[gg]
        assert {s.qcfg for s in shapes} == {"w4a16_g-1_asym", "w8a8_g-1_sym"}
        hps = [HostProblem(s.M, s.N, s.K, QParams(s.a_bits, s.w_bits, s.gsize, s.sym), seed=500 + i, device=DEV)
               for i, s in enumerate(shapes)]
        GroupGemm([h.problem for h in hps], variant=variant).launch()
        torch.cuda.synchronize()
        for h in hps:
            if h.M == 0:
                continue
            rows = np.unique(rng.integers(0, h.M, size=min(h.M, 16)))
            cols = np.unique(rng.integers(0, h.N, size=24))
            out = h.result()[np.ix_(rows, cols)]
            ref = h.expected()[np.ix_(rows, cols)]
            if h.q.is_weight_only:
                assert_f16_close(out, ref, h.K)
            else:
                assert (out.view(np.uint16) == ref.view(np.uint16)).all(), f"{gg} w8a8 M={h.M}"


@pytest.mark.parametrize("variant", WO)
@pytest.mark.parametrize("bits", [2, 4, 8])
def test_wo3_group_sizes_scale_slots_and_row_skip(bits, variant):
    """wo3's round-4 loop (gg_tile_wo under kWo3): scale groups of 1 / 2 / 4 / 8 stages (g64 opens a
    group at every stage: a scale DMA beside every ring buffer), sym and asym, experts of 1-63 rows
    (row blocks past M skipped), a multi-m-tile problem, and a long-K low-fill call the planner
    splits along K (scale groups crossing slice boundaries; write-through split-K hand-off)."""
    specs = [(35, 512, 1024, 64, True), (17, 256, 2048, 64, False), (49, 768, 1536, 128, True),
             (1, 256, 1024, 256, False), (63, 512, 2048, 512, True), (130, 264, 1024, 256, False),
             (33, 256, 5632, 64, False), (64, 128, 4096, 128, True)]
    hps = [HostProblem(M, N, K, QParams(16, bits, g, s), seed=900 + i, device=DEV)
           for i, (M, N, K, g, s) in enumerate(specs)]
    group_gemm([h.problem for h in hps], variant=variant)
    torch.cuda.synchronize()
    _check(hps)
