"""CHECK mode of the CLI (the role of test.cu's CaseMode::CHECK, test.cu:725-729 / test_utils.h:70-95).

Recomputes a random sample of rows x columns of every problem on the CPU with torch (C[rows, cols]
depends only on A[rows] and B[cols]), for every quant type the library runs:

  * wxax per channel (w8a8 / w4a4 g-1): unpacked pack_wxax codes, exact int64 dot products, the
    reference epilogue fp16_rn(0 + f32(acc) * f32(fp16_rn(sa * sb))) (mm_tile.cuh:469-496) — bit exact;
  * wxax grouped (w4a4 g128): scales [K/g][M] / [K/g][N] (permute_scale, quantize.cuh:299-315); per
    group out = fma(f32(acc_g), f32(fp16_rn(sa_g * sb_g)), out), C = fp16_rn(out)
    (cta_gemm.cuh:610-772) — bit exact (the fma formed in f64, where product and sum are exact);
  * weight-only WxA16: B codes unpacked from the kernel layout, dequantised exactly as the kernels
    do, fp16(fma(u - off, scale, zp)) (quantize.cuh:146-213), then an f64 GEMM — fp16 tolerance;
  * w8a8 E4M3: e4m3 codes decoded, exact f64 dot products rounded to f32, the wxax epilogue — fp16
    tolerance (the MFMA's f32 summation order is unspecified);
  * fp16 / bf16: f64 GEMM — relative 1e-3 (north_star) with a cancellation floor.

Unlike the reference's CHECK (abs tol 1.0 against an unquantised cutlass GEMM), integer paths must
match bit for bit.
"""
from __future__ import annotations

import numpy as np
import torch

from .quantize import dequant_weightonly, unpack_wxax, unpack_weightonly_mi355x


def _f16_close(out: torch.Tensor, ref: torch.Tensor, what: str) -> None:
    err = (out.double() - ref).abs()
    tol = 1e-3 * ref.abs() + 1e-3 * ref.pow(2).mean().sqrt() + 1e-6
    if not torch.isfinite(out).all() or (err > tol).any():
        raise AssertionError(f"CHECK failed: {what}: max err {err.max().item()}")


def _bit_exact(out: torch.Tensor, ref: torch.Tensor, what: str) -> None:
    if not torch.equal(out.view(torch.int16), ref.view(torch.int16)):
        bad = (out.view(torch.int16) != ref.view(torch.int16)).sum().item()
        raise AssertionError(f"CHECK failed: {what}: {bad} outputs differ")


def expected_sample(p, rows: torch.Tensor, cols: torch.Tensor) -> tuple[torch.Tensor, bool]:
    """Reference values of C[rows][:, cols] for one problem (CPU) and whether they are bit-exact."""
    q = p.q
    A = p.A.index_select(0, rows).cpu()
    if q.is_weight_only:
        codes = unpack_weightonly_mi355x(p.B.index_select(0, cols).cpu(), q.w_bits, p.K)
        G = 1 if q.gsize == -1 else p.K // q.gsize
        sz = p.scale_b.cpu().reshape(G, p.N, -1).index_select(1, cols.cpu()).reshape(-1)
        Bdq = dequant_weightonly(codes, sz, q.w_bits, q.gsize, q.sym)
        return A.double() @ Bdq.double().T, False
    if not q.is_quant:
        return A.double() @ p.B.index_select(0, cols).cpu().double().T, False
    if q.is_fp8:
        def dec(t):
            return unpack_wxax(t, 8, p.K).view(torch.float8_e4m3fn).double()
        acc = (dec(A) @ dec(p.B.index_select(0, cols).cpu()).T).float()
        sa = p.scale_a.index_select(0, rows).cpu().float()
        sb = p.scale_b.index_select(0, cols).cpu().float()
        s16 = (sa[:, None] * sb[None, :]).half().float()
        return (0.0 + acc * s16).half().double(), False
    qa = unpack_wxax(A, q.a_bits, p.K).to(torch.int64)
    qb = unpack_wxax(p.B.index_select(0, cols).cpu(), q.w_bits, p.K).to(torch.int64)
    if q.gsize == -1:
        sa = p.scale_a.index_select(0, rows).cpu().float()
        sb = p.scale_b.index_select(0, cols).cpu().float()
        s16 = (sa[:, None] * sb[None, :]).half().float()
        return (0.0 + (qa @ qb.T).float() * s16).half(), True
    G = p.K // q.gsize
    sa = p.scale_a.cpu().reshape(G, p.M).index_select(1, rows.cpu()).float()
    sb = p.scale_b.cpu().reshape(G, p.N).index_select(1, cols.cpu()).float()
    out = torch.zeros(len(rows), len(cols), dtype=torch.float32)
    for g in range(G):
        ks = slice(g * q.gsize, (g + 1) * q.gsize)
        acc = qa[:, ks] @ qb[:, ks].T
        s16 = (sa[g][:, None] * sb[g][None, :]).half().double()
        out = (acc.double() * s16 + out.double()).float()  # f64: product and sum exact -> one rounding
    return out.half(), True


def check_sampled(problems, n: int = 32, seed: int = 0) -> None:
    rng = np.random.default_rng(seed)
    for p in problems:
        if p.M == 0 or p.N == 0:
            continue
        rows = torch.from_numpy(np.sort(rng.choice(p.M, min(n, p.M), replace=False))).to(p.C.device)
        cols = torch.from_numpy(np.sort(rng.choice(p.N, min(n, p.N), replace=False))).to(p.C.device)
        out = p.C.index_select(0, rows).index_select(1, cols).cpu()
        ref, exact = expected_sample(p, rows, cols)
        what = f"{p.q.qcfg} M={p.M} N={p.N} K={p.K}"
        if exact:
            _bit_exact(out, ref, what)
        else:
            _f16_close(out, ref, what)
