"""CPU oracle for the weight-only WxA16 branches — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.

Restates, in numpy, the reference's weight-only data preparation and arithmetic:
  * ``quant_wo``: ``quant_weight`` (mxmoe/kernels/src/include/quantize.cuh:218-279) applied per
    (column, group) as the harness does (test.cu:325-336, one "row" per group of ``gsize`` K values):
    sym: scale = max(|min|, |max|) / qmax, zp = 0, q in [-qmax, qmax]; asym: zp = min,
    scale = (max - min) / (2^bits - 1), q in [0, 2^bits - 1]; scale 0 -> 1; fp16 arithmetic,
    q = round-half-even(clamp((w - zp) / scale)). (The harness passes ``a_bits`` = 16 as the code
    width, test.cu:335 — a reference bug; the intended ``w_bits`` is used here.)
  * ``permute_scale`` (quantize.cuh:297-315): [N][G](x2) -> [G][N](x2).
  * ``stored_codes``: the values ``pack_weightonly`` writes (quantize.cuh:387-421): sym codes are
    offset by 2^(bits-1) - 1 "for fast dequant", asym codes as they are.
  * ``ref_pack``: ``permute_weight`` (Row mode, quantize.cuh:318-385) followed by
    ``pack_weightonly`` — the reference's packed B bytes, fed to ``mxmoe_gg_repack_weightonly``.
  * ``dequant``: the B value the reference's mainloop multiplies (cta_gemm.cuh:112-286 with
    ``Converter::dequant_frag``, quantize.cuh:146-213): fp16(fma(u - off, scale, zp)), one rounding,
    with off = 2^(bits-1) - 1 for sym. (The reference's 8- and 2-bit converters skip the sym offset,
    quantize.cuh:150-154; the intended arithmetic is used.)
  * ``gemm``: C = fp16(A . B_deq^T) accumulated in f64 (the reference accumulates the fp16 MMA in
    f32, so parity is the fp16 tolerance of tests/_util.py).
"""
from __future__ import annotations

import numpy as np


def qrange(bits: int, sym: bool) -> tuple[int, int]:
    return (-((1 << (bits - 1)) - 1), (1 << (bits - 1)) - 1) if sym else (0, (1 << bits) - 1)


def sym_offset(bits: int, sym: bool) -> int:
    return (1 << (bits - 1)) - 1 if sym else 0


def quant_wo(w: np.ndarray, bits: int, gsize: int, sym: bool) -> tuple[np.ndarray, np.ndarray]:
    """fp16 [N, K] -> (codes int32 [N, K], scale_zp fp16 in the reference quant_weight layout:
    sym [N*G], asym [N*G, 2] with row n*G + g)."""
    assert w.dtype == np.float16
    N, K = w.shape
    g = K if gsize == -1 else gsize
    assert K % g == 0
    grp = w.reshape(N * (K // g), g)
    lo, hi = grp.min(axis=1), grp.max(axis=1)
    lower, upper = qrange(bits, sym)
    up = np.float16(upper)
    if sym:
        zp = np.zeros_like(lo)
        scale = (np.maximum(np.abs(lo), np.abs(hi)) / up).astype(np.float16)
    else:
        zp = lo
        scale = ((hi - lo).astype(np.float16) / up).astype(np.float16)
    scale = np.where(scale == 0, np.float16(1), scale).astype(np.float16)
    qv = ((grp - zp[:, None]).astype(np.float16) / scale[:, None]).astype(np.float16)
    qv = np.clip(qv, np.float16(lower), up)
    q = np.rint(qv.astype(np.float32)).astype(np.int32)  # rint = round half to even
    sz = scale if sym else np.stack([scale, zp], axis=1)
    return q.reshape(N, K), sz


def permute_scale(sz: np.ndarray, N: int, K: int, gsize: int, sym: bool) -> np.ndarray:
    """quant_weight layout [N*G](x2) -> kernel layout [G][N](x2) (flattened fp16)."""
    G = 1 if gsize == -1 else K // gsize
    if sym:
        return np.ascontiguousarray(sz.reshape(N, G).T).reshape(-1)
    return np.ascontiguousarray(sz.reshape(N, G, 2).transpose(1, 0, 2)).reshape(-1)


def stored_codes(q: np.ndarray, bits: int, sym: bool) -> np.ndarray:
    return (q + sym_offset(bits, sym)).astype(np.int32)


def _perm_indices(bits: int) -> np.ndarray:
    """intermediate_perm of permute_weight (compose_perm_indices, quantize.cuh:283-295)."""
    if bits == 8:
        proj, desired, plen = [1, 0, 3, 2], [0, 2, 4, 6, 1, 3, 5, 7], 4
    elif bits == 4:
        proj, desired, plen = [3, 7, 2, 6, 1, 5, 0, 4], [0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15], 8
    elif bits == 2:
        proj = [7, 15, 6, 14, 5, 13, 4, 12, 3, 11, 2, 10, 1, 9, 0, 8]
        desired = [0, 8, 16, 24, 1, 9, 17, 25, 2, 10, 18, 26, 3, 11, 19, 27,
                   4, 12, 20, 28, 5, 13, 21, 29, 6, 14, 22, 30, 7, 15, 23, 31]
        plen = 16
    else:
        raise ValueError(bits)
    n = len(desired)
    perm = [0] * n
    for i in range(0, n, plen):
        for j in range(plen):
            perm[proj[j] + i] = desired[i + j]
    return np.array(perm)


def permute_weight(w: np.ndarray, bits: int) -> np.ndarray:
    """permute_weight(PermuteMode::Row) on codes [N, K] (column-major weight of the reference)."""
    N, K = w.shape
    pack = 16 // bits
    assert N % (pack * 8) == 0 and K % 16 == 0
    perm = _perm_indices(bits)
    flat = w.reshape(-1)
    res = np.empty_like(flat)
    for j in range(0, N, pack * 8):
        for i in range(0, K, 16):
            for trav_j in range(8):
                for trav_i in range(0, 8, 2):
                    idx = [(i + ii + trav_i + trav_ii) + (j + f * 8 + trav_j) * K
                           for ii in (0, 8) for trav_ii in (0, 1) for f in range(pack)]
                    vals = flat[idx]
                    res[idx] = vals[perm]
    return res.reshape(N, K)


def pack_weightonly(w: np.ndarray, bits: int) -> np.ndarray:
    """pack_weightonly on (already offset) codes [N, K] -> uint16 words [N/PACK, K]."""
    N, K = w.shape
    pack = 16 // bits
    out = np.zeros((N // pack, K), dtype=np.uint16)
    mask = (1 << bits) - 1
    for j in range(0, N, pack * 8):
        for jj in range(8):
            v = np.zeros(K, dtype=np.uint32)
            for f in range(pack):
                v = (v << bits) | (w[j + f * 8 + jj].astype(np.uint32) & mask)
            out[j // pack + jj] = v.astype(np.uint16)
    return out


def ref_pack(q: np.ndarray, bits: int, sym: bool) -> np.ndarray:
    """The reference's packed B for codes q (what its harness would hand the kernel)."""
    return pack_weightonly(permute_weight(stored_codes(q, bits, sym), bits), bits)


def mi355x_pack(q: np.ndarray, bits: int, sym: bool) -> np.ndarray:
    """The layout libmxmoe_gg consumes (include/mxmoe_gg.h): per 64-K segment of a row, unit g of
    K values {kc*32 + g*8 + e} stored at element position g*16 + kc*8 + e; 4-bit: e at nibble
    (e >> 1) | (e & 1) << 2 of the unit (codes 2q, 2q+1 at bits 4q, 16 + 4q), low nibble first."""
    N, K = q.shape
    u = stored_codes(q, bits, sym).astype(np.uint8).reshape(N, K // 64, 2, 4, 8).transpose(0, 1, 3, 2, 4)
    if bits == 2:  # unit (seg, g): one little-endian 32-bit word, code (kc, e) at bit 16 (e&1) + 2 (4 kc + e//2)
        kc, e = np.meshgrid(np.arange(2), np.arange(8), indexing="ij")
        shift = (e % 2) * 16 + 2 * (4 * kc + e // 2)
        word = (u.astype(np.uint64) << shift.astype(np.uint64)).sum(axis=(-2, -1)).astype(np.uint32)
        return np.ascontiguousarray(word).view(np.uint8).reshape(N, K // 4)
    if bits == 8:
        return np.ascontiguousarray(u.reshape(N, K))
    assert bits == 4
    u = u[..., [0, 2, 4, 6, 1, 3, 5, 7]].reshape(N, K)
    return (u[:, 0::2] | (u[:, 1::2] << 4)).astype(np.uint8)


def dequant(q: np.ndarray, sz_kernel: np.ndarray, N: int, K: int, bits: int, gsize: int, sym: bool) -> np.ndarray:
    """B_deq fp16 [N, K] = fp16(fma(q, scale, zp)) with the kernel-layout scales [G][N](x2)."""
    G = 1 if gsize == -1 else K // gsize
    g = K if gsize == -1 else gsize
    if sym:
        s = sz_kernel.reshape(G, N).T.astype(np.float64)
        z = np.zeros_like(s)
    else:
        t = sz_kernel.reshape(G, N, 2).transpose(1, 0, 2).astype(np.float64)
        s, z = t[..., 0], t[..., 1]
    s = np.repeat(s, g, axis=1)
    z = np.repeat(z, g, axis=1)
    return (q.astype(np.float64) * s + z).astype(np.float16)  # exact in f64, one rounding


def gemm(A: np.ndarray, Bdq: np.ndarray) -> np.ndarray:
    return (A.astype(np.float64) @ Bdq.astype(np.float64).T).astype(np.float16)
