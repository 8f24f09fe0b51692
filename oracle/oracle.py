"""Python wrapper of the CPU oracle (``oracle/gg_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker. The product path (mxmoe_amd) never imports this module.

Every function restates reference arithmetic (SeaCatComplexes/MxMoE):
  quant_rtn_sym ....... quantize.cuh:218-279 (quant_weight), quant.py:40-84 (quant_minmax)
  pack / unpack ....... quantize.cuh:425-475 (pack_wxax)
  gg_quant ............ cta_gemm.cuh:423-608 + mm_tile.cuh:469-496, 610-662
  gg_quant_grouped .... cta_gemm.cuh:610-772 (w4a4 g128: per-group int32 dot products, fmaf fold)
  gg_f16 .............. cta_gemm.cuh:7-107 (f64 accumulate here; tolerance-checked)
  gg_bf16 ............. the same with bfloat16 operands (MMA_BF16_FP32, tile_config.py:64-102)
  quant_e4m3 / gg_e4m3 . w8a8_g-1_sym_E4M3 (tile_config.py:45, 192; cuda_utils.cuh:385-410): the
                         reference has no E4M3 quantiser or codegen branch, so the quantiser is this
                         repo's definition (parity unpinned by the reference; e4m3 codes pinned to
                         torch.float8_e4m3fn)
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "lib" / "libgg_oracle.so"

_lib = None


def build() -> Path:
    subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = ctypes.CDLL(str(LIB_PATH))
        c = ctypes
        P = c.c_void_p
        _lib.oracle_f16_to_f32.restype = c.c_float
        _lib.oracle_f16_to_f32.argtypes = [c.c_uint16]
        _lib.oracle_f32_to_f16.restype = c.c_uint16
        _lib.oracle_f32_to_f16.argtypes = [c.c_float]
        _lib.oracle_pack_wxax.argtypes = [P, P, c.c_int64, c.c_int64, c.c_int]
        _lib.oracle_unpack_wxax.argtypes = [P, P, c.c_int64, c.c_int64, c.c_int]
        _lib.oracle_quant_rtn_sym.argtypes = [P, P, P, c.c_int64, c.c_int64, c.c_int]
        _lib.oracle_gg_quant.argtypes = [P, P, P, P, P, c.c_int64, c.c_int64, c.c_int64, c.c_int, c.c_int64,
                                         c.c_int64, c.c_int64, c.c_int]
        _lib.oracle_gg_quant_grouped.argtypes = [P, P, P, P, P, c.c_int64, c.c_int64, c.c_int64, c.c_int, c.c_int64,
                                                 c.c_int64, c.c_int64, c.c_int64, c.c_int]
        _lib.oracle_gg_f16.argtypes = [P, P, P, c.c_int64, c.c_int64, c.c_int64, c.c_int64, c.c_int64, c.c_int64,
                                       c.c_int]
        _lib.oracle_e4m3_to_f32.restype = c.c_float
        _lib.oracle_e4m3_to_f32.argtypes = [c.c_uint8]
        _lib.oracle_f32_to_e4m3.restype = c.c_uint8
        _lib.oracle_f32_to_e4m3.argtypes = [c.c_float]
        _lib.oracle_quant_e4m3.argtypes = [P, P, P, c.c_int64, c.c_int64]
        _lib.oracle_gg_e4m3.argtypes = [P, P, P, P, P, c.c_int64, c.c_int64, c.c_int64, c.c_int64, c.c_int64,
                                        c.c_int64, c.c_int]
        _lib.oracle_gg_bf16.argtypes = [P, P, P, c.c_int64, c.c_int64, c.c_int64, c.c_int64, c.c_int64, c.c_int64,
                                        c.c_int]
        _lib.oracle_max_threads.restype = c.c_int
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed with {rc}")


def max_threads() -> int:
    return lib().oracle_max_threads()


def quant_rtn_sym(x_f16: np.ndarray, bits: int) -> tuple[np.ndarray, np.ndarray]:
    x = np.ascontiguousarray(x_f16, dtype=np.float16)
    rows, K = x.shape
    q = np.empty((rows, K), np.int8)
    s = np.empty((rows,), np.float16)
    _chk(lib().oracle_quant_rtn_sym(_p(x), _p(q), _p(s), rows, K, bits), "quant")
    return q, s


def quant_rtn_sym_grouped(x_f16: np.ndarray, bits: int, gsize: int) -> tuple[np.ndarray, np.ndarray]:
    """quant_weight over [rows * K/gsize] blocks of gsize K elements (test.cu:240-284), then
    permute_scale (quantize.cuh:299-315): codes [rows, K], scales [K/gsize * rows] group-major."""
    x = np.ascontiguousarray(x_f16, dtype=np.float16)
    rows, K = x.shape
    q, s = quant_rtn_sym(x.reshape(rows * (K // gsize), gsize), bits)
    return q.reshape(rows, K), np.ascontiguousarray(s.reshape(rows, K // gsize).T).reshape(-1)


def pack_wxax(q: np.ndarray, bits: int) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.int8)
    rows, K = q.shape
    out = np.empty((rows, K * bits // 8), np.uint8)
    _chk(lib().oracle_pack_wxax(_p(q), _p(out), rows, K, bits), "pack")
    return out


def unpack_wxax(p: np.ndarray, bits: int, K: int) -> np.ndarray:
    p = np.ascontiguousarray(p, dtype=np.uint8)
    q = np.empty((p.shape[0], K), np.int8)
    _chk(lib().oracle_unpack_wxax(_p(p), _p(q), p.shape[0], K, bits), "unpack")
    return q


def gg_quant(A: np.ndarray, B: np.ndarray, sa: np.ndarray, sb: np.ndarray, M: int, N: int, K: int, bits: int,
             threads: int = 0) -> np.ndarray:
    """Expected fp16 C [M,N] of one w8a8 / w4a4 problem from packed A [M,K*bits/8], B [N,K*bits/8]."""
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    sa = np.ascontiguousarray(sa, np.float16)
    sb = np.ascontiguousarray(sb, np.float16)
    C = np.zeros((M, N), np.float16)
    kb = K * bits // 8
    _chk(lib().oracle_gg_quant(_p(A), _p(B), _p(sa), _p(sb), _p(C), M, N, K, bits, kb, kb, N, threads), "gg_quant")
    return C


def gg_quant_grouped(A: np.ndarray, B: np.ndarray, sa: np.ndarray, sb: np.ndarray, M: int, N: int, K: int,
                     bits: int, gsize: int, threads: int = 0) -> np.ndarray:
    """Expected fp16 C [M,N] of one group-quantised (w4a4 g128) problem; sa [K/g][M], sb [K/g][N]."""
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    sa = np.ascontiguousarray(sa, np.float16)
    sb = np.ascontiguousarray(sb, np.float16)
    C = np.zeros((M, N), np.float16)
    kb = K * bits // 8
    _chk(lib().oracle_gg_quant_grouped(_p(A), _p(B), _p(sa), _p(sb), _p(C), M, N, K, bits, gsize, kb, kb, N, threads),
         "gg_quant_grouped")
    return C


def gg_f16(A: np.ndarray, B: np.ndarray, M: int, N: int, K: int, threads: int = 0) -> np.ndarray:
    A = np.ascontiguousarray(A, np.float16)
    B = np.ascontiguousarray(B, np.float16)
    C = np.zeros((M, N), np.float16)
    _chk(lib().oracle_gg_f16(_p(A), _p(B), _p(C), M, N, K, K, K, N, threads), "gg_f16")
    return C


def quant_e4m3(x_f16: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Per-row E4M3: (uint8 e4m3 codes [rows, K] in logical order, fp16 scales [rows])."""
    x = np.ascontiguousarray(x_f16, dtype=np.float16)
    rows, K = x.shape
    q = np.empty((rows, K), np.uint8)
    s = np.empty((rows,), np.float16)
    _chk(lib().oracle_quant_e4m3(_p(x), _p(q), _p(s), rows, K), "quant_e4m3")
    return q, s


def e4m3_to_f32(codes: np.ndarray) -> np.ndarray:
    lut = np.array([lib().oracle_e4m3_to_f32(i) for i in range(256)], np.float32)
    return lut[np.asarray(codes, np.uint8)]


def f32_to_e4m3(x: np.ndarray) -> np.ndarray:
    f = lib().oracle_f32_to_e4m3
    return np.array([f(float(v)) for v in np.asarray(x, np.float32).ravel()], np.uint8).reshape(np.shape(x))


def gg_e4m3(A: np.ndarray, B: np.ndarray, sa: np.ndarray, sb: np.ndarray, M: int, N: int, K: int,
            threads: int = 0) -> np.ndarray:
    """Expected fp16 C [M,N] of one w8a8 E4M3 problem from A [M,K], B [N,K] code bytes (pack_wxax order)."""
    A = np.ascontiguousarray(A, np.uint8)
    B = np.ascontiguousarray(B, np.uint8)
    sa = np.ascontiguousarray(sa, np.float16)
    sb = np.ascontiguousarray(sb, np.float16)
    C = np.zeros((M, N), np.float16)
    _chk(lib().oracle_gg_e4m3(_p(A), _p(B), _p(sa), _p(sb), _p(C), M, N, K, K, K, N, threads), "gg_e4m3")
    return C


def gg_bf16(A: np.ndarray, B: np.ndarray, M: int, N: int, K: int, threads: int = 0) -> np.ndarray:
    """Expected fp16 C [M,N] of one bf16 problem; A [M,K], B [N,K] as uint16 bfloat16 bit patterns."""
    A = np.ascontiguousarray(A, np.uint16)
    B = np.ascontiguousarray(B, np.uint16)
    C = np.zeros((M, N), np.float16)
    _chk(lib().oracle_gg_bf16(_p(A), _p(B), _p(C), M, N, K, K, K, N, threads), "gg_bf16")
    return C


def acc_exact(qa: np.ndarray, qb: np.ndarray) -> np.ndarray:
    """Exact integer accumulator sum_k qa[m,k]*qb[n,k] (int64, numpy) — used by property tests."""
    return qa.astype(np.int64) @ qb.astype(np.int64).T


def epilogue(acc: np.ndarray, sa: np.ndarray, sb: np.ndarray) -> np.ndarray:
    """fp16_rn(0 + f32(acc) * f32(fp16_rn(sa[m]*sb[n]))) (mm_tile.cuh:490-493, 642-645)."""
    s16 = (sa.astype(np.float32)[:, None] * sb.astype(np.float32)[None, :]).astype(np.float16)
    v = np.float32(0.0) + acc.astype(np.float32) * s16.astype(np.float32)
    return v.astype(np.float16)


if __name__ == "__main__":  # pragma: no cover
    print(build(), os.path.getsize(LIB_PATH))
