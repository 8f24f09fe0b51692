"""Input preparation for quantised GroupGEMM problems (bench / test setup — not the hot path).

Weight-only (WxA16) inputs: ``quant_weightonly`` restates the reference's ``quant_weight``
(quantize.cuh:218-279) per (column, group) in fp16 (sym: scale = max|w| / qmax, zp = 0;
asym: zp = min, scale = (max - min) / (2^bits - 1)), returning the codes as ``pack_weightonly``
stores them (sym offset by 2^(bits-1) - 1) and scale / zp in the reference ``permute_scale``
layout; ``pack_weightonly_mi355x`` writes the kernel layout documented at
``mxmoe_gg_repack_weightonly`` (include/mxmoe_gg.h). Reference-packed weights go through
``_native.repack_weightonly`` instead.

Restates, in torch (runs on CPU or on the GPU for the bs=8192 shapes):
  * ``quant_rtn_sym``: RTN per-row symmetric quantisation in fp16, the reference's
    ``quant_weight`` kernel (mxmoe/kernels/src/include/quantize.cuh:218-279) and
    ``quant_minmax`` (mxmoe/quant/quant.py:40-84): scale = fp16(max|x| / qmax) (0 -> 1),
    q = round_half_even(clamp(fp16(x / scale), -qmax, qmax)).
  * ``pack_wxax``: the 16-bit word packing of ``pack_wxax`` (quantize.cuh:425-475): element
    j+x of a word sits at bits (PACK-1-x)*bits (first element in the HIGH bits), two's complement
    fields, little-endian words.  int8: byte[2j] = q[2j+1], byte[2j+1] = q[2j];
    int4: byte[2j] = (q[4j+2] << 4) | q[4j+3], byte[2j+1] = (q[4j] << 4) | q[4j+1].
"""
from __future__ import annotations

import torch


def qmax_of(bits: int) -> int:
    return (1 << (bits - 1)) - 1


def quant_rtn_sym(x: torch.Tensor, bits: int, gsize: int = -1) -> tuple[torch.Tensor, torch.Tensor]:
    """Symmetric RTN of an fp16 [rows, K] tensor -> (int8 codes [rows, K], fp16 scales).

    gsize -1: one scale per row, scale [rows].  gsize g: one scale per (row, g-element K group), the
    reference harness's quant_weight over [rows * K/g] blocks (test.cu:240-284) followed by
    permute_scale (quantize.cuh:299-315): scale [K/g * rows], group-major ([K/g][rows])."""
    if x.dtype != torch.float16:
        raise TypeError("quant_rtn_sym expects fp16 input (the reference quantises in half)")
    if bits not in (4, 8):
        raise ValueError("only 4/8-bit WxAx quantisation is supported")
    rows, K = x.shape
    g = K if gsize == -1 else gsize
    if g <= 0 or K % g:
        raise ValueError(f"K={K} must be a multiple of the group size {gsize}")
    qmax = qmax_of(bits)
    grp = x.reshape(rows, K // g, g)
    amax = grp.abs().amax(dim=-1)
    scale = amax / qmax  # fp16 / int -> fp16, correctly rounded
    scale = torch.where(scale == 0, torch.ones_like(scale), scale)
    q = (grp / scale[..., None]).clamp(-qmax, qmax).round()  # round = half to even
    q = q.to(torch.int8).reshape(rows, K)
    if gsize == -1:
        return q, scale.reshape(rows)
    return q, scale.t().contiguous().reshape(-1)


def pack_wxax(q: torch.Tensor, bits: int) -> torch.Tensor:
    """int8 codes [rows, K] -> packed bytes uint8 [rows, K*bits/8] (reference pack_wxax layout)."""
    rows, K = q.shape
    if bits == 8:
        if K % 2:
            raise ValueError("pack_dim not aligned with pack_num")
        w = q.reshape(rows, K // 2, 2)
        out = torch.stack([w[..., 1], w[..., 0]], dim=-1)
        return out.reshape(rows, K).view(torch.uint8)
    if bits == 4:
        if K % 4:
            raise ValueError("pack_dim not aligned with pack_num")
        n = (q.to(torch.int16) & 0xF).reshape(rows, K // 4, 4)
        b0 = (n[..., 2] << 4) | n[..., 3]
        b1 = (n[..., 0] << 4) | n[..., 1]
        return torch.stack([b0, b1], dim=-1).reshape(rows, K // 2).to(torch.uint8)
    raise ValueError("only support [4, 8] bits sym quantization")


def unpack_wxax(p: torch.Tensor, bits: int, K: int) -> torch.Tensor:
    """Inverse of pack_wxax: packed bytes -> int8 codes [rows, K] in logical order."""
    rows = p.shape[0]
    if bits == 8:
        w = p.view(torch.int8).reshape(rows, K // 2, 2)
        return torch.stack([w[..., 1], w[..., 0]], dim=-1).reshape(rows, K)
    if bits == 4:
        b = p.to(torch.int16).reshape(rows, K // 4, 2)
        b0, b1 = b[..., 0], b[..., 1]
        nib = torch.stack([(b1 >> 4) & 0xF, b1 & 0xF, (b0 >> 4) & 0xF, b0 & 0xF], dim=-1)
        nib = torch.where(nib >= 8, nib - 16, nib)
        return nib.reshape(rows, K).to(torch.int8)
    raise ValueError("only support [4, 8] bits")


E4M3_MAX = 448.0  # largest finite OCP e4m3 value


def quant_e4m3(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row E4M3 quantisation of fp16 [rows, K] for w8a8_g-1_sym_E4M3 -> (uint8 OCP e4m3 codes in
    logical K order, fp16 scales [rows]): scale = fp16(amax / 448), 1 for an all-zero row and at
    least 2^-14 (the smallest normal fp16: a tiny row keeps nonzero codes instead of flushing to a
    zero or subnormal scale), code = e4m3_rn(f32(x) / f32(scale)), saturating. The reference defines the strategy (QCFG_W8A8_E4M3, tile_config.py:192)
    but ships no quantiser for it; this is the natural per-channel analogue of quant_weight
    (quantize.cuh:218-279), restated in oracle/gg_oracle.c (oracle_quant_e4m3)."""
    if x.dtype != torch.float16:
        raise TypeError("quant_e4m3 expects fp16 input")
    amax = x.abs().amax(dim=-1).float()
    scale = (amax / E4M3_MAX).half().clamp_min(2.0 ** -14)
    scale = torch.where(amax == 0, torch.ones_like(scale), scale)
    q = (x.float() / scale.float()[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), scale


def pack_e4m3(codes: torch.Tensor) -> torch.Tensor:
    """uint8 e4m3 codes [rows, K] -> the pack_wxax 8-bit byte order (QCFG_W8A8_E4M3: T_PACK half,
    PACK_DIM K — each 16-bit word holds elements (2j, 2j+1) with 2j in the high byte)."""
    return pack_wxax(codes.view(torch.int8), 8)


def quantize_pack(x: torch.Tensor, bits: int) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp16 [rows, K] -> (packed uint8, fp16 scale, int8 codes)."""
    q, s = quant_rtn_sym(x, bits)
    return pack_wxax(q, bits), s, q


def quant_weightonly(w: torch.Tensor, bits: int, gsize: int, sym: bool) -> tuple[torch.Tensor, torch.Tensor]:
    """fp16 [N, K] -> (stored codes uint8 [N, K], scale_zp fp16 flat: sym [G][N], asym [G][N][2])."""
    if w.dtype != torch.float16:
        raise TypeError("quant_weightonly expects fp16 input (the reference quantises in half)")
    if bits not in (2, 4, 8):
        raise ValueError("weight-only: 2 / 4 / 8-bit codes")
    N, K = w.shape
    g = K if gsize == -1 else gsize
    if K % g:
        raise ValueError("K must be a multiple of the group size")
    grp = w.reshape(N, K // g, g)
    lo, hi = grp.amin(dim=-1), grp.amax(dim=-1)
    if sym:
        qmax = (1 << (bits - 1)) - 1
        lower, upper = -qmax, qmax
        zp = torch.zeros_like(lo)
        scale = torch.maximum(lo.abs(), hi.abs()) / upper
    else:
        lower, upper = 0, (1 << bits) - 1
        zp = lo
        scale = (hi - lo) / upper
    scale = torch.where(scale == 0, torch.ones_like(scale), scale)
    q = ((grp - zp[..., None]) / scale[..., None]).clamp(lower, upper).round()  # half-to-even
    codes = (q.to(torch.int16) + ((1 << (bits - 1)) - 1 if sym else 0)).to(torch.uint8).reshape(N, K)
    if sym:
        sz = scale.t().contiguous().reshape(-1)
    else:
        sz = torch.stack([scale, zp], dim=-1).transpose(0, 1).contiguous().reshape(-1)
    return codes, sz


def pack_weightonly_mi355x(codes: torch.Tensor, bits: int) -> torch.Tensor:
    """Stored codes uint8 [N, K] -> kernel layout uint8 [N, K * bits / 8]: in each 64-K segment the
    K values {kc*32 + g*8 + e} sit at element position g*16 + kc*8 + e (4-bit: e at nibble
    (e >> 1) | (e & 1) << 2 of the unit, include/mxmoe_gg.h); 4-bit low nibble first; 2-bit: the
    unit's 16 codes in one little-endian 32-bit word."""
    N, K = codes.shape
    if K % 64:
        raise ValueError("weight-only needs K % 64 == 0")
    if bits == 2:  # unit (seg, g) = one 32-bit word: code (kc, e) at bit 16 (e & 1) + 2 (4 kc + e // 2)
        e = torch.arange(8)
        shift = ((e % 2) * 16)[None, :] + 2 * (4 * torch.arange(2)[:, None] + e[None, :] // 2)
        u = codes.reshape(N, K // 64, 2, 4, 8).to(torch.int64).transpose(2, 3)  # [N, seg, g, kc, e]
        word = (u << shift.to(codes.device)).sum(dim=(-2, -1)).to(torch.int32)  # [N, seg, g]
        return word.contiguous().view(torch.uint8).reshape(N, K // 4)
    u = codes.reshape(N, K // 64, 2, 4, 8).transpose(2, 3)
    if bits == 8:
        return u.reshape(N, K).contiguous()
    u = u[..., [0, 2, 4, 6, 1, 3, 5, 7]].reshape(N, K)
    return (u[:, 0::2] | (u[:, 1::2] << 4)).contiguous()


def unpack_weightonly_mi355x(packed: torch.Tensor, bits: int, K: int) -> torch.Tensor:
    """Inverse of pack_weightonly_mi355x: kernel layout uint8 [N, K * bits / 8] -> stored codes uint8 [N, K]."""
    N = packed.shape[0]
    if K % 64:
        raise ValueError("weight-only needs K % 64 == 0")
    if bits == 2:
        word = packed.contiguous().view(torch.int32).reshape(N, K // 64, 4).to(torch.int64)
        e = torch.arange(8)
        shift = (((e % 2) * 16)[None, :] + 2 * (4 * torch.arange(2)[:, None] + e[None, :] // 2)).to(packed.device)
        u = (word[..., None, None] >> shift) & 3  # [N, seg, g, kc, e]
        return u.transpose(2, 3).reshape(N, K).to(torch.uint8)
    if bits == 8:
        return packed.reshape(N, K // 64, 4, 2, 8).transpose(2, 3).reshape(N, K).contiguous()
    if bits != 4:
        raise ValueError("weight-only: 2 / 4 / 8-bit codes")
    lo, hi = packed & 0xF, packed >> 4
    u = torch.stack([lo, hi], dim=-1).reshape(N, K // 64, 4, 2, 8)  # [N, seg, g, kc, stored position]
    inv = torch.tensor([0, 4, 1, 5, 2, 6, 3, 7], device=packed.device)  # position p holds e = [0,2,4,6,1,3,5,7][p]
    u = u.index_select(-1, inv)
    return u.transpose(2, 3).reshape(N, K).contiguous()


def dequant_weightonly(codes: torch.Tensor, sz: torch.Tensor, bits: int, gsize: int, sym: bool) -> torch.Tensor:
    """Stored codes uint8 [N, K] + kernel-layout scale_zp ([G][N] sym, [G][N][2] asym) -> the fp16 B the
    kernels multiply: fp16(fma(u - off, scale, zp)), one rounding (Converter::dequant_frag,
    quantize.cuh:146-213; off = 2^(bits-1) - 1 for sym codes, pack_weightonly quantize.cuh:387-421)."""
    N, K = codes.shape
    G = 1 if gsize == -1 else K // gsize
    g = K if gsize == -1 else gsize
    if sym:
        s = sz.reshape(G, N).t().double()
        z = torch.zeros_like(s)
    else:
        t = sz.reshape(G, N, 2).transpose(0, 1).double()
        s, z = t[..., 0], t[..., 1]
    off = (1 << (bits - 1)) - 1 if sym else 0
    u = codes.to(torch.float64).reshape(N, G, g) - off
    return (u * s[..., None] + z[..., None]).reshape(N, K).half()  # exact in f64, then one rounding
