"""CHECK mode of the CLI (the role of test.cu's CaseMode::CHECK, test.cu:725-729 / test_utils.h:70-95).

Recomputes a random sample of rows x columns of every problem on the CPU with torch: unpacked
codes, exact int64 accumulation and the reference epilogue (mm_tile.cuh:469-496) for quantised
problems; f64 matmul for fp16. Unlike the reference's CHECK (abs tol 1.0 against an unquantised
cutlass GEMM), quantised problems must match bit for bit and fp16 within 1e-3 relative.
"""
from __future__ import annotations

import numpy as np
import torch

from .quantize import unpack_wxax


def check_sampled(problems, n: int = 32, seed: int = 0) -> None:
    rng = np.random.default_rng(seed)
    for p in problems:
        if p.M == 0 or p.N == 0:
            continue
        rows = torch.from_numpy(np.sort(rng.choice(p.M, min(n, p.M), replace=False))).to(p.C.device)
        cols = torch.from_numpy(np.sort(rng.choice(p.N, min(n, p.N), replace=False))).to(p.C.device)
        out = p.C.index_select(0, rows).index_select(1, cols).cpu()
        A = p.A.index_select(0, rows).cpu()
        B = p.B.index_select(0, cols).cpu()
        if p.q.is_quant:
            qa = unpack_wxax(A, p.q.a_bits, p.K).to(torch.int64)
            qb = unpack_wxax(B, p.q.w_bits, p.K).to(torch.int64)
            acc = qa @ qb.T
            sa = p.scale_a.index_select(0, rows).cpu().float()
            sb = p.scale_b.index_select(0, cols).cpu().float()
            s16 = (sa[:, None] * sb[None, :]).half().float()
            ref = (0.0 + acc.float() * s16).half()
            if not torch.equal(out.view(torch.int16), ref.view(torch.int16)):
                bad = (out.view(torch.int16) != ref.view(torch.int16)).sum().item()
                raise AssertionError(f"CHECK failed: {p.q.qcfg} M={p.M} N={p.N} K={p.K}: {bad} outputs differ")
        else:
            ref = A.double() @ B.double().T
            err = (out.double() - ref).abs()
            tol = 1e-3 * ref.abs() + 1e-3 * ref.pow(2).mean().sqrt() + 1e-6
            if (err > tol).any():
                raise AssertionError(f"CHECK failed: fp16 M={p.M} N={p.N} K={p.K}: max err {err.max().item()}")
