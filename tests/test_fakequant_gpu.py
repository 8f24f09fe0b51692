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


@pytest.mark.parametrize("ref_format", [False, True], ids=["mi355x_layout", "reference_packed_repack"])
def test_weightonly_hip_matches_reference_fake_quant(ref_format):
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
    group_gemm(probs)
    torch.cuda.synchronize()
    for p, r in zip(probs, refs):
        assert_fakequant_close(p.C[: p.M, : p.N].cpu().numpy(), r, f"{p.q.qcfg} M={p.M} N={p.N} K={p.K}")
