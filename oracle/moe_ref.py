"""CPU restatement of the MoE-layer plumbing (include/mxmoe_moe.h) — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker. It restates, in numpy + the C oracle:
  route ............. torch::sort(topk_ids.view(-1)) / floor_divide(topk) / bincount(E)
                      (ref_bind.cu:47-64, 452-456), stable sort
  quant_act ......... hidden rows gathered in slot order (index_select, ref_bind.cu:57), each
                      expert's rows quantised by its tag (cvt_qparams_to_tag, :467-479) with the
                      reference quant_weight (quantize.cuh:218-279; oracle.quant_rtn_sym[_grouped])
                      and packed by pack_wxax (quantize.cuh:425-475)
  silu_mul .......... act = fp16(f32(silu(f32 g)) * f32 u): the reference's silu_mul_then_quant_kernel
                      lives in the missing act_kernel.cuh, so this arithmetic is "parity unpinned"
                      (our definition; exp is libm's expf here, the GPU uses the hardware v_exp_f32 /
                      v_rcp_f32 approximations: a few f32 ulps apart, i.e. at most 1 fp16 ulp / 1 code
                      step after rounding, which the tests tolerate)
  combine ........... acc = fma(w_k, y_k, acc) over k in order, then fma(shared_w, shared, acc), fp16
                      (gg_unpermute_out is an empty stub in the reference, :66: our definition)
"""
from __future__ import annotations

import numpy as np

from oracle import oracle

ACT_FP16, ACT_INT8, ACT_INT4, ACT_INT4_G128 = 0, 1, 2, 3


def route(topk_ids: np.ndarray, E: int):
    flat = topk_ids.reshape(-1).astype(np.int64)
    order = np.argsort(flat, kind="stable")
    topk = topk_ids.shape[1]
    sorted_e = flat[order].astype(np.int32)
    perm = (order // topk).astype(np.int32)
    inv = np.empty_like(order)
    inv[order] = np.arange(order.size)
    counts = np.bincount(flat, minlength=E).astype(np.int32)
    return sorted_e, perm, inv.astype(np.int32), counts


def quant_rows(x: np.ndarray, tag: int):
    """fp16 rows [R, W] -> (stored bytes [R, W*bits/8] or fp16 rows, scales or None)."""
    if tag == ACT_FP16:
        return x.astype(np.float16), None
    if tag == ACT_INT4_G128:
        q, s = oracle.quant_rtn_sym_grouped(x, 4, 128)
        return oracle.pack_wxax(q, 4), s
    bits = 8 if tag == ACT_INT8 else 4
    q, s = oracle.quant_rtn_sym(x, bits)
    return oracle.pack_wxax(q, bits), s


def silu_mul(gu: np.ndarray) -> np.ndarray:
    """fp16 [R, 2N] (gate | up) -> fp16 [R, N]."""
    N = gu.shape[1] // 2
    g = gu[:, :N].astype(np.float32)
    u = gu[:, N:].astype(np.float32)
    with np.errstate(over="ignore"):
        s = g / (np.float32(1) + np.exp(-g, dtype=np.float32))
    return (s * u).astype(np.float16)


def fma_f32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """fmaf elementwise: the f64 product of f32 x fp16-valued operands is exact; the f64 sum is checked
    exact (TwoSum) so the single f32 rounding below is the fma's."""
    p = a.astype(np.float64) * b.astype(np.float64)
    o = c.astype(np.float64)
    t = p + o
    bp = t - o
    err = (p - bp) + (o - (t - bp))
    assert (err == 0).all(), "f64 sum inexact: fma restatement would double-round"
    return t.astype(np.float32)


def combine(y: np.ndarray, inv: np.ndarray, w: np.ndarray, topk: int, shared=None, shared_w=None) -> np.ndarray:
    T = w.shape[0]
    acc = np.zeros((T, y.shape[1]), np.float32)
    for k in range(topk):
        acc = fma_f32(w[:, k:k + 1].astype(np.float32), y[inv.reshape(T, topk)[:, k]], acc)
    if shared is not None:
        sw = np.ones((T, 1), np.float32) if shared_w is None else shared_w.reshape(T, 1).astype(np.float32)
        acc = fma_f32(sw, shared, acc)
    return acc.astype(np.float16)
