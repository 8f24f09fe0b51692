"""Weight-only WxA16 GroupGEMM on the GPU vs the oracle (fp16 tolerance of tests/_util.py)."""
from __future__ import annotations

import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import FP16, W4A4, W8A8, GroupGemm, QParams, group_gemm
from tests._util import HostProblem, assert_f16_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
V2 = [int(ln.split()[0]) for ln in nat.list_variants() if ln.split()[1].startswith("v2")]
QS = [QParams(16, b, g, s) for b in (2, 4, 8) for g in (-1, 128) for s in (True, False)]


def _check(hps):
    for hp in hps:
        if hp.M:
            assert_f16_close(hp.result(), hp.expected(), hp.K)


@pytest.mark.parametrize("variant", V2)
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
