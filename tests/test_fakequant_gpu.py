"""HIP GroupGEMM output vs the reference's executed fake-quant linear (tests/golden/gg_fakequant_ref.npz).

Same inputs as the committed vectors, every production variant; tolerance and its rationale:
tests/_util.assert_fakequant_close. The bit-exact comparison against the C oracle stays in
tests/test_golden_gpu.py; this one anchors the result on code the reference itself ran
(Quantizer.fake_quant + F.linear, mxmoe/quant/quant.py:87-106).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import Problem, QParams, group_gemm
from oracle import weightonly
from tests._util import assert_fakequant_close
from tests.test_fakequant_ref import KINDS, quant_problems, wo_problems

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("variant", nat.production_variants())
@pytest.mark.parametrize("kind", list(KINDS))
def test_hip_matches_reference_fake_quant(kind, variant):
    probs, refs = [], []
    for i, M, N, K, bits, gsize, d, cfq in quant_problems(kind):
        C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=DEV)
        probs.append(Problem(A=torch.from_numpy(d[f"p{i}_A"]).to(DEV), B=torch.from_numpy(d[f"p{i}_B"]).to(DEV),
                             C=C, M=M, N=N, K=K, q=QParams(bits, bits, gsize, True),
                             scale_a=torch.from_numpy(d[f"p{i}_sa"]).to(DEV),
                             scale_b=torch.from_numpy(d[f"p{i}_sb"]).to(DEV)))
        refs.append(cfq)
    if kind == "w4a4g128" and not nat.variant_supports(variant, "w4a4_g128_sym"):
        pytest.skip("variant has no w4a4_g128 tile body")
    group_gemm(probs, variant=variant)
    torch.cuda.synchronize()
    for p, r in zip(probs, refs):
        assert_fakequant_close(p.C[: p.M, : p.N].cpu().numpy(), r, f"{kind} M={p.M} N={p.N} K={p.K}")


@pytest.mark.parametrize("variant", [None] + nat.production_variants("w4a16_g-1_asym"))  # None: AUTO
@pytest.mark.parametrize("ref_format", [False, True], ids=["mi355x_layout", "reference_packed_repack"])
def test_weightonly_hip_matches_reference_fake_quant(ref_format, variant):
    probs, refs = [], []
    for i, M, N, K, bits, gsize, sym, fq in wo_problems():
        q, sz = weightonly.quant_wo(fq[f"wo{i}_B"], bits, gsize, sym)  # == the reference's quant_minmax
        if ref_format:
            B = nat.repack_weightonly(weightonly.ref_pack(q, bits, sym), N, K, bits)
        else:
            B = weightonly.mi355x_pack(q, bits, sym)
        C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=DEV)
        probs.append(Problem(A=torch.from_numpy(fq[f"wo{i}_A"]).to(DEV), B=torch.from_numpy(B).to(DEV), C=C,
                             M=M, N=N, K=K, q=QParams(16, bits, gsize, sym),
                             scale_b=torch.from_numpy(weightonly.permute_scale(sz, N, K, gsize, sym)).to(DEV)))
        refs.append(fq[f"wo{i}_Cfq"])
    group_gemm(probs, variant=variant)
    torch.cuda.synchronize()
    for p, r in zip(probs, refs):
        assert_fakequant_close(p.C[: p.M, : p.N].cpu().numpy(), r, f"{p.q.qcfg} M={p.M} N={p.N} K={p.K}")


def _w4a16_w8a8_problems():
    """The reference's hand-instantiated small-batch pairing (hz_fused.cuh:14-125: w4a16_g-1_asym +
    w8a8_g-1_sym in one fused kernel): the fixture's w8a8 problems and its w4a16 g-1 asym problems."""
    probs, refs, exact = [], [], []
    for i, M, N, K, bits, gsize, d, cfq in quant_problems("w8a8"):
        C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=DEV)
        probs.append(Problem(A=torch.from_numpy(d[f"p{i}_A"]).to(DEV), B=torch.from_numpy(d[f"p{i}_B"]).to(DEV),
                             C=C, M=M, N=N, K=K, q=QParams(8, 8, -1, True),
                             scale_a=torch.from_numpy(d[f"p{i}_sa"]).to(DEV),
                             scale_b=torch.from_numpy(d[f"p{i}_sb"]).to(DEV)))
        refs.append(cfq)
        exact.append(d[f"p{i}_C"])
    n_wo = 0
    for i, M, N, K, bits, gsize, sym, fq in wo_problems():
        if (bits, gsize, sym) != (4, -1, False):
            continue
        q, sz = weightonly.quant_wo(fq[f"wo{i}_B"], bits, gsize, sym)
        C = torch.full((max(M, 1), N), float("nan"), dtype=torch.float16, device=DEV)
        probs.append(Problem(A=torch.from_numpy(fq[f"wo{i}_A"]).to(DEV),
                             B=torch.from_numpy(weightonly.mi355x_pack(q, bits, sym)).to(DEV), C=C, M=M, N=N, K=K,
                             q=QParams(16, 4, -1, False),
                             scale_b=torch.from_numpy(weightonly.permute_scale(sz, N, K, gsize, sym)).to(DEV)))
        refs.append(fq[f"wo{i}_Cfq"])
        exact.append(None)
        n_wo += 1
    assert n_wo >= 1 and len(probs) > n_wo
    return probs, refs, exact


@pytest.mark.parametrize("variant", [v for v in nat.production_variants("w4a16_g-1_asym")
                                     if nat.variant_supports(v, "w8a8_g-1_sym")])
def test_w4a16_w8a8_fused_launch_matches_reference_fake_quant(variant):
    probs, refs, exact = _w4a16_w8a8_problems()
    group_gemm(probs, variant=variant)
    torch.cuda.synchronize()
    for p, r, e in zip(probs, refs, exact):
        out = p.C[: p.M, : p.N].cpu().numpy()
        assert_fakequant_close(out, r, f"{p.q.qcfg} M={p.M} N={p.N} K={p.K}")
        if e is not None:  # w8a8: also bit-exact against the C oracle's committed output
            assert (out.view(np.uint16) == e.view(np.uint16)).all(), f"w8a8 M={p.M}"
