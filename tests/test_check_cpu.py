"""CLI CHECK mode (mxmoe_amd/check.py) on CPU tensors: for every quant type, a C filled with the
oracle's expected output passes and a single corrupted sampled element fails (weight-only
and g128 problems used to crash or compare against wrong scales)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from mxmoe_amd.check import check_sampled
from mxmoe_amd.groupgemm import FP16, W4A4, W4A4_G128, W8A8, QParams
from tests._util import HostProblem

QS = [FP16, W8A8, W4A4, W4A4_G128] + [QParams(16, b, g, s) for b in (2, 4, 8) for g in (-1, 128) for s in (True, False)]


@pytest.mark.parametrize("q", QS, ids=[q.qcfg for q in QS])
def test_check_accepts_oracle_output_and_rejects_corruption(q):
    hp = HostProblem(40, 136 if q.is_weight_only or not q.is_quant else 128, 256, q, seed=5, device="cpu")
    hp.problem.C[: hp.M, : hp.N] = torch.from_numpy(hp.expected())
    check_sampled([hp.problem], n=hp.N)  # every column, up to 136 rows: the whole problem
    c = hp.problem.C
    c[3, 7] = c[3, 7] * 2 + 1
    with pytest.raises(AssertionError, match="CHECK failed"):
        check_sampled([hp.problem], n=hp.N)


def test_slice_problem_scales_every_layout():
    """harness.slice_problem: columns [n0, n1) of per-channel, grouped and weight-only problems."""
    from mxmoe_amd.harness import slice_problem

    for q in QS:
        if not q.is_quant:
            continue
        hp = HostProblem(9, 384, 256, q, seed=11, device="cpu")
        p = hp.problem
        s = slice_problem(p, 128, 384)
        G = 1 if q.gsize == -1 else 256 // q.gsize
        full = p.scale_b.reshape(G, 384, -1)
        assert torch.equal(s.scale_b.reshape(G, 256, -1), full[:, 128:384]), q.qcfg
        assert s.scale_b.is_contiguous() and s.N == 256 and s.B.shape[0] == 256
        if q.is_quant and not q.is_weight_only:
            assert torch.equal(s.scale_a, p.scale_a)


def test_slice_rows_scales_every_layout():
    """harness.slice_rows (the expert split's shared-expert row slices): rows [m0, m1) of A, C and
    the per-row scales — per-channel [M] as a view, w4a4 g128 [K/128][M] as a copy of [:, m0:m1]."""
    from mxmoe_amd.harness import slice_rows

    for q in QS:
        hp = HostProblem(200, 128, 256, q, seed=12, device="cpu")
        p = hp.problem
        s = slice_rows(p, 64, 192)
        assert s.M == 128 and torch.equal(s.A, p.A[64:192]) and s.C.data_ptr() == p.C[64:].data_ptr()
        if p.scale_a is None:
            assert s.scale_a is None
            continue
        G = 1 if q.gsize == -1 else 256 // q.gsize
        assert torch.equal(s.scale_a.reshape(G, 128), p.scale_a.reshape(G, 200)[:, 64:192]), q.qcfg
        assert s.scale_a.is_contiguous() and s.scale_b is p.scale_b
        C = torch.zeros(128, 128, dtype=torch.float16)
        assert slice_rows(p, 64, 192, C=C).C is C
