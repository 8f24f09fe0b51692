/*
 * gg_oracle.c — CPU restatement of the reference GroupGEMM arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline — never as the product path.
 *
 * Restates (SeaCatComplexes/MxMoE, read as text; the CUDA sources cannot be built here):
 *   quant_weight  RTN per-row sym in fp16 ............ mxmoe/kernels/src/include/quantize.cuh:218-279
 *   pack_wxax     16-bit word packing (first element in the high bits) ... quantize.cuh:425-475
 *   w8a8/w4a4     exact integer dot product over K ... cta_gemm.cuh:423-608 (int32 mma accumulate)
 *   epilogue      out = fp16_rn(0 + f32(acc) * f32(fp16_rn(sa[m]*sb[n])))
 *                 ............................... mm_tile.cuh:469-496 (scale_frag), 610-662 (store)
 *   w4a4 g128     per-group int32 dot products folded with fmaf ... cta_gemm.cuh:610-772
 *   fp16          C = fp16_rn(sum_k a*b) with an f64 accumulator (the reference accumulates in
 *                 f32 on tensor cores, order unspecified: cta_gemm.cuh:7-107) — tolerance-checked.
 *   bf16          the same with bfloat16 operands (MMA_BF16_FP32, tile_config.py:64-102).
 *   w8a8 E4M3     OCP fp8 e4m3 operands (QCFG_W8A8_E4M3 tile_config.py:192: T_PACK half, PACK_DIM K,
 *                 i.e. pack_wxax byte order; mma m16n8k32 e4m3 -> f32, cuda_utils.cuh:385-410), the
 *                 products exact and summed exactly here (f64), then the wxax epilogue on f32(acc)
 *                 (mm_tile.cuh:469-496). The reference ships no E4M3 quantiser and no codegen branch
 *                 for it (compose_kernel.py:47-57): the quantiser below (per-row scale amax/448,
 *                 one RNE rounding to e4m3, saturating) is this repo's definition — parity unpinned
 *                 by the reference; the code <-> value map is pinned to torch.float8_e4m3fn in tests.
 * The column-scale index uses the INTENDED sb[n] (SURVEY.md §8(a) a11 documents the reference's
 * lane%4 indexing bug; tests/golden also holds the bug-compatible permuted-scale variant).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- IEEE binary16 <-> binary32, round-to-nearest-even, subnormals kept ---- */
float oracle_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ff;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else { /* subnormal: normalise */
      int e = -1;
      do {
        e++;
        man <<= 1;
      } while ((man & 0x400) == 0);
      bits = sign | ((uint32_t)(127 - 15 - e) << 23) | ((man & 0x3ff) << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp - 15 + 127) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

uint16_t oracle_f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) { /* inf / nan */
    return (uint16_t)(sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u | ((absx >> 13) & 0x3ffu) : 0));
  }
  if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
  if (absx < 0x38800000u) {                                     /* result subnormal or zero */
    if (absx < 0x33000000u) return (uint16_t)sign;              /* < 2^-25: rounds to 0 */
    uint32_t e = absx >> 23;
    uint32_t m = (absx & 0x7fffffu) | 0x800000u;
    /* value = m * 2^(e-150); subnormal unit 2^-24 -> q = m * 2^(e-126) = m >> (126-e) */
    uint32_t shift = 126 - e; /* 14..24 */
    uint32_t q = m >> shift;
    uint32_t rem = m & ((1u << shift) - 1);
    uint32_t halfway = 1u << (shift - 1);
    if (rem > halfway || (rem == halfway && (q & 1))) q++;
    return (uint16_t)(sign | q);
  }
  uint32_t e = (absx >> 23) - 127 + 15;
  uint32_t m = absx & 0x7fffffu;
  uint32_t q = (e << 10) | (m >> 13);
  uint32_t rem = m & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (q & 1))) q++;
  return (uint16_t)(sign | q);
}

/* fp16 x fp16 -> fp16 (RN). The f32 product of two binary16 values is exact. */
static uint16_t f16_mul(uint16_t a, uint16_t b) { return oracle_f32_to_f16(oracle_f16_to_f32(a) * oracle_f16_to_f32(b)); }

/* ---- pack_wxax (quantize.cuh:425-475): element j+x of a 16-bit word at bits (PACK-1-x)*bits,
 *      stored little-endian.  q: int8 [rows][K] logical codes; out: bytes [rows][K*bits/8]. ---- */
int oracle_pack_wxax(const int8_t* q, uint8_t* out, int64_t rows, int64_t K, int bits) {
  if (bits != 8 && bits != 4) return -1;
  const int pack = 16 / bits;
  if (K % pack) return -2;
  const int64_t wpr = K / pack; /* words per row */
  for (int64_t r = 0; r < rows; ++r) {
    for (int64_t w = 0; w < wpr; ++w) {
      uint16_t v = 0;
      for (int x = 0; x < pack; ++x) {
        int val = q[r * K + w * pack + x];
        uint16_t field = bits == 8 ? (uint16_t)(uint8_t)(((val < 0) << 7) | (val & 0x7f))
                                   : (uint16_t)(((val < 0) << 3) | (val & 0x7));
        v = (uint16_t)((v << bits) | field);
      }
      out[r * wpr * 2 + 2 * w] = (uint8_t)(v & 0xff);
      out[r * wpr * 2 + 2 * w + 1] = (uint8_t)(v >> 8);
    }
  }
  return 0;
}

/* inverse of pack_wxax for one row: packed bytes -> logical int8 codes */
static void unpack_row(const uint8_t* p, int8_t* q, int64_t K, int bits) {
  const int pack = 16 / bits;
  for (int64_t w = 0; w < K / pack; ++w) {
    uint16_t v = (uint16_t)(p[2 * w] | ((uint16_t)p[2 * w + 1] << 8));
    for (int x = 0; x < pack; ++x) {
      int sh = (pack - 1 - x) * bits;
      int f = (v >> sh) & ((1 << bits) - 1);
      if (f & (1 << (bits - 1))) f -= (1 << bits);
      q[w * pack + x] = (int8_t)f;
    }
  }
}

int oracle_unpack_wxax(const uint8_t* packed, int8_t* q, int64_t rows, int64_t K, int bits) {
  if (bits != 8 && bits != 4) return -1;
  const int64_t rb = K * bits / 8;
  for (int64_t r = 0; r < rows; ++r) unpack_row(packed + r * rb, q + r * K, K, bits);
  return 0;
}

/* ---- quant_weight (quantize.cuh:218-279), sym per-row (gsize -1), all arithmetic in fp16:
 *      scale = fp16(max(|min|,|max|) / qmax), 0 -> 1;  q = rint_even(clamp(fp16(x/scale), +-qmax)) ---- */
int oracle_quant_rtn_sym(const uint16_t* x, int8_t* q, uint16_t* scale, int64_t rows, int64_t K, int bits) {
  if (bits != 8 && bits != 4) return -1;
  const float qmax = (float)((1 << (bits - 1)) - 1);
  for (int64_t r = 0; r < rows; ++r) {
    float mx = 0.0f;
    for (int64_t k = 0; k < K; ++k) {
      float v = fabsf(oracle_f16_to_f32(x[r * K + k]));
      if (v > mx) mx = v;
    }
    uint16_t s = oracle_f32_to_f16(mx / qmax); /* f32 division of two halves, then RN to half */
    if ((s & 0x7fff) == 0) s = 0x3c00;         /* scale == 0 -> 1 */
    scale[r] = s;
    float sf = oracle_f16_to_f32(s);
    for (int64_t k = 0; k < K; ++k) {
      float d = oracle_f16_to_f32(oracle_f32_to_f16(oracle_f16_to_f32(x[r * K + k]) / sf));
      if (d > qmax) d = qmax;
      if (d < -qmax) d = -qmax;
      q[r * K + k] = (int8_t)nearbyintf(d); /* __half2int_rn: round half to even */
    }
  }
  return 0;
}

/* ---- w8a8 / w4a4 GroupGEMM problem: C[m][n] (row stride ldc elements) ----
 * A: packed bytes [M][lda_b], B: packed bytes [N][ldb_b]; the sum over k is formed exactly
 * (int32 is exact: |acc| <= 128*128*K < 2^31 for K <= 131072). */
int oracle_gg_quant(const uint8_t* A, const uint8_t* B, const uint16_t* sa, const uint16_t* sb, uint16_t* C,
                    int64_t M, int64_t N, int64_t K, int bits, int64_t lda_b, int64_t ldb_b, int64_t ldc,
                    int nthreads) {
  if (bits != 8 && bits != 4) return -1;
  if (K > 131072) return -2;
  int8_t* bq = (int8_t*)malloc((size_t)(N * K > 0 ? N * K : 1));
  if (!bq) return -3;
  for (int64_t n = 0; n < N; ++n) unpack_row(B + n * ldb_b, bq + n * K, K, bits);
  int rc = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t m = 0; m < M; ++m) {
    int8_t* aq = (int8_t*)malloc((size_t)(K > 0 ? K : 1));
    if (!aq) {
      rc = -3;
      continue;
    }
    unpack_row(A + m * lda_b, aq, K, bits);
    for (int64_t n = 0; n < N; ++n) {
      const int8_t* b = bq + n * K;
      int32_t acc = 0;
      for (int64_t k = 0; k < K; ++k) acc += (int32_t)aq[k] * (int32_t)b[k];
      const uint16_t s16 = f16_mul(sa[m], sb[n]);
      const float v = 0.0f + (float)acc * oracle_f16_to_f32(s16);
      C[m * ldc + n] = oracle_f32_to_f16(v);
    }
    free(aq);
  }
  free(bq);
  return rc;
}

/* ---- w4a4 g128 (group-quantised WxAx) problem: cta_gemm_w4a4g128, cta_gemm.cuh:610-772 ----
 * Per group g of `gsize` K elements an exact int32 dot product acc_g, folded in group order into an
 * f32 accumulator: out = fmaf(f32(acc_g), f32(fp16_rn(sa[g][m] * sb[g][n])), out), starting from
 * +0 (frag_c_out{} then `frag_out += T(acc) * T(sa * sb)`, mm_tile.cuh:490-493 — nvcc's default
 * --fmad contracts that into one FFMA); C = fp16_rn(out) (mm_tile.cuh:642-645).
 * sa: [K/gsize][M], sb: [K/gsize][N] (permute_scale layout, quantize.cuh:299-315). */
int oracle_gg_quant_grouped(const uint8_t* A, const uint8_t* B, const uint16_t* sa, const uint16_t* sb, uint16_t* C,
                            int64_t M, int64_t N, int64_t K, int bits, int64_t gsize, int64_t lda_b, int64_t ldb_b,
                            int64_t ldc, int nthreads) {
  if (bits != 8 && bits != 4) return -1;
  if (gsize <= 0 || K % gsize) return -2;
  const int64_t G = K / gsize;
  int8_t* bq = (int8_t*)malloc((size_t)(N * K > 0 ? N * K : 1));
  if (!bq) return -3;
  for (int64_t n = 0; n < N; ++n) unpack_row(B + n * ldb_b, bq + n * K, K, bits);
  int rc = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t m = 0; m < M; ++m) {
    int8_t* aq = (int8_t*)malloc((size_t)(K > 0 ? K : 1));
    if (!aq) {
      rc = -3;
      continue;
    }
    unpack_row(A + m * lda_b, aq, K, bits);
    for (int64_t n = 0; n < N; ++n) {
      const int8_t* b = bq + n * K;
      float out = 0.0f;
      for (int64_t g = 0; g < G; ++g) {
        int32_t acc = 0;
        for (int64_t k = g * gsize; k < (g + 1) * gsize; ++k) acc += (int32_t)aq[k] * (int32_t)b[k];
        const uint16_t s16 = f16_mul(sa[g * M + m], sb[g * N + n]);
        out = fmaf((float)acc, oracle_f16_to_f32(s16), out);
      }
      C[m * ldc + n] = oracle_f32_to_f16(out);
    }
    free(aq);
  }
  free(bq);
  return rc;
}

/* ---- OCP fp8 e4m3 (e4m3fn: bias 7, no infinities, S.1111.111 = NaN, max 448) ---- */
float oracle_e4m3_to_f32(uint8_t v) {
  const int e = (v >> 3) & 15, m = v & 7;
  float mag;
  if (e == 15 && m == 7) return (v & 0x80) ? -NAN : NAN;
  if (e == 0) mag = ldexpf((float)m, -9); /* subnormal: m * 2^-3 * 2^-6 */
  else mag = ldexpf(1.0f + (float)m / 8.0f, e - 7);
  return (v & 0x80) ? -mag : mag;
}

/* f32 -> e4m3, round to nearest even, saturating to +-448 (NaN -> NaN) */
uint8_t oracle_f32_to_e4m3(float f) {
  if (f != f) return 0x7f;
  const uint8_t sign = signbit(f) ? 0x80 : 0;
  float a = fabsf(f);
  if (a >= 448.0f) return sign | 0x7e;
  /* candidates: every non-negative finite code is monotone in its value; pick the nearest, ties even */
  int lo = 0, hi = 0x7e;
  while (hi - lo > 1) { /* largest code with value <= a */
    const int mid = (lo + hi) / 2;
    if (oracle_e4m3_to_f32((uint8_t)mid) <= a) lo = mid;
    else hi = mid;
  }
  if (oracle_e4m3_to_f32((uint8_t)hi) <= a) lo = hi;
  if (lo == 0x7e) return sign | 0x7e;
  const float vlo = oracle_e4m3_to_f32((uint8_t)lo), vhi = oracle_e4m3_to_f32((uint8_t)(lo + 1));
  const double dlo = (double)a - vlo, dhi = (double)vhi - a;
  int q = lo;
  if (dhi < dlo || (dhi == dlo && (lo & 1))) q = lo + 1;
  return sign | (uint8_t)q;
}

/* per-row E4M3 quantisation of fp16 x: scale = fp16(amax / 448) (0 -> 1), q = e4m3_rn(f32(x) / f32(scale)) */
int oracle_quant_e4m3(const uint16_t* x, uint8_t* q, uint16_t* scale, int64_t rows, int64_t K) {
  for (int64_t r = 0; r < rows; ++r) {
    float mx = 0.0f;
    for (int64_t k = 0; k < K; ++k) {
      float v = fabsf(oracle_f16_to_f32(x[r * K + k]));
      if (v > mx) mx = v;
    }
    uint16_t s = oracle_f32_to_f16(mx / 448.0f);
    if (mx == 0.0f) s = 0x3c00;           /* all-zero row: scale 1 */
    else if (s < 0x0400) s = 0x0400;      /* at least the smallest normal fp16, 2^-14 */
    scale[r] = s;
    const float sf = oracle_f16_to_f32(s);
    for (int64_t k = 0; k < K; ++k) q[r * K + k] = oracle_f32_to_e4m3(oracle_f16_to_f32(x[r * K + k]) / sf);
  }
  return 0;
}

/* ---- w8a8 E4M3 GroupGEMM problem: A [M][lda_b], B [N][ldb_b] bytes in pack_wxax byte order
 *      (byte 2j holds element 2j+1 and vice versa; the same order on A and B, so the byte-wise dot
 *      product is the element-wise one). acc = f32(exact sum), C = fp16_rn(0 + acc * f32(fp16_rn(sa*sb))). */
int oracle_gg_e4m3(const uint8_t* A, const uint8_t* B, const uint16_t* sa, const uint16_t* sb, uint16_t* C,
                   int64_t M, int64_t N, int64_t K, int64_t lda_b, int64_t ldb_b, int64_t ldc, int nthreads) {
  float lut[256];
  for (int i = 0; i < 256; ++i) lut[i] = oracle_e4m3_to_f32((uint8_t)i);
  int rc = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t m = 0; m < M; ++m) {
    for (int64_t n = 0; n < N; ++n) {
      const uint8_t* a = A + m * lda_b;
      const uint8_t* b = B + n * ldb_b;
      double acc = 0.0; /* products of e4m3 values have <= 8 significant bits: exact in f64 */
      for (int64_t k = 0; k < K; ++k) acc += (double)lut[a[k]] * (double)lut[b[k]];
      const uint16_t s16 = f16_mul(sa[m], sb[n]);
      const float v = 0.0f + (float)acc * oracle_f16_to_f32(s16);
      C[m * ldc + n] = oracle_f32_to_f16(v);
    }
  }
  return rc;
}

/* ---- bf16 GroupGEMM problem (f64 accumulate, RN to fp16). A [M][lda], B [N][ldb] in elements. ---- */
int oracle_gg_bf16(const uint16_t* A, const uint16_t* B, uint16_t* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                   int64_t ldb, int64_t ldc, int nthreads) {
  int rc = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t m = 0; m < M; ++m) {
    for (int64_t n = 0; n < N; ++n) {
      double acc = 0.0;
      for (int64_t k = 0; k < K; ++k) {
        uint32_t ab = (uint32_t)A[m * lda + k] << 16, bb = (uint32_t)B[n * ldb + k] << 16;
        float af, bf;
        memcpy(&af, &ab, 4);
        memcpy(&bf, &bb, 4);
        acc += (double)af * (double)bf;
      }
      C[m * ldc + n] = oracle_f32_to_f16((float)acc);
    }
  }
  return rc;
}

/* ---- fp16 GroupGEMM problem (f64 accumulate, RN to fp16). A [M][lda], B [N][ldb] in elements. ---- */
int oracle_gg_f16(const uint16_t* A, const uint16_t* B, uint16_t* C, int64_t M, int64_t N, int64_t K, int64_t lda,
                  int64_t ldb, int64_t ldc, int nthreads) {
  float* bf = (float*)malloc((size_t)(N * K > 0 ? N * K : 1) * sizeof(float));
  if (!bf) return -3;
  for (int64_t n = 0; n < N; ++n)
    for (int64_t k = 0; k < K; ++k) bf[n * K + k] = oracle_f16_to_f32(B[n * ldb + k]);
  int rc = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t m = 0; m < M; ++m) {
    float* af = (float*)malloc((size_t)(K > 0 ? K : 1) * sizeof(float));
    if (!af) {
      rc = -3;
      continue;
    }
    for (int64_t k = 0; k < K; ++k) af[k] = oracle_f16_to_f32(A[m * lda + k]);
    for (int64_t n = 0; n < N; ++n) {
      const float* b = bf + n * K;
      double acc = 0.0;
      for (int64_t k = 0; k < K; ++k) acc += (double)af[k] * (double)b[k];
      C[m * ldc + n] = oracle_f32_to_f16((float)acc);
    }
    free(af);
  }
  free(bf);
  return rc;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
