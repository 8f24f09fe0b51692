// Probe (lab, not product): can gfx950's block-scaled fp6 MFMA carry the w4a4 int4 x int4 dot
// product exactly, and at what issue rate against the int8 MFMA the int4 tiles use today?
//   * int4 v in [-8, 7] encoded as FP6 E3M2 (fmt 3, bias 3: every integer up to 8 is exact) with
//     unit E8M0 scales, or as E2M3 (fmt 2) of v / 2 with scales 2^1 (max 7.5 needs the halving);
//   * one 16x16x128 MFMA against an int64 host product under the lane map assumed below, then a
//     K = 14336 chain of worst-case (-8 x -8) products (917504: exact if the f32 adds are);
//   * issue rate: 4 independent accumulators, 4096 MFMAs per wave, 8 waves per CU x 1024 CUs.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/probe_f6 tools/probe_f6.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int32_t v8i __attribute__((ext_vector_type(8)));
typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint32_t code_e3m2(int v) {  // sign | exp(3, bias 3) | mant(2)
  static const uint32_t mag[9] = {0, 12, 16, 18, 20, 21, 22, 23, 24};
  return (v < 0 ? 32u : 0u) | mag[v < 0 ? -v : v];
}
static uint32_t code_e2m3(int v) {  // v / 2: sign | exp(2, bias 1) | mant(3)
  static const uint32_t mag[9] = {0, 4, 8, 12, 16, 18, 20, 22, 24};
  return (v < 0 ? 32u : 0u) | mag[v < 0 ? -v : v];
}
// 32 six-bit codes -> 6 dwords, code j at bits [6j, 6j + 6) of the 192-bit little-endian word
static void pack32(const uint32_t* codes, uint32_t* out) {
  memset(out, 0, 24);
  for (int j = 0; j < 32; ++j) {
    const int bit = 6 * j;
    out[bit / 32] |= codes[j] << (bit % 32);
    if (bit % 32 > 26) out[bit / 32 + 1] |= codes[j] >> (32 - bit % 32);
  }
}

template <int FMT>
__global__ void one_mfma(const uint32_t* a6, const uint32_t* b6, float* c, int scale, int reps) {
  const int l = threadIdx.x;
  v8i a = {0, 0, 0, 0, 0, 0, 0, 0}, b = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int d = 0; d < 6; ++d) { a[d] = a6[l * 6 + d]; b[d] = b6[l * 6 + d]; }
  v4f acc = {0, 0, 0, 0};
  for (int r = 0; r < reps; ++r)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, FMT, FMT, 0, scale, 0, scale);
  for (int i = 0; i < 4; ++i) c[l * 4 + i] = acc[i];
}

// issue rate: 4 independent chains per wave
template <int KIND>
__global__ __launch_bounds__(512) void rate(float* sink, int iters) {
  const int l = threadIdx.x;
  v8i a = {l, l + 1, l + 2, l + 3, l + 4, l + 5, 0, 0};
  v4f f[4] = {};
  v4i q[4] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (KIND == 0) f[u] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, f[u], 3, 3, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      else if constexpr (KIND == 1) q[u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(v4i{a[0], a[1], a[2], a[3]}, v4i{a[4], a[5], a[0], a[1]}, q[u], 0, 0, 0);
      else f[u] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, f[u], 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    }
  }
  float s = 0;
  for (int u = 0; u < 4; ++u) s += f[u][0] + f[u][3] + (float)q[u][0] + (float)q[u][3];
  if (s == 1234.5f) sink[l] = s;
}

int main() {
  // ---- one MFMA, random ints, both formats ----
  srand(7);
  int A[16][128], B[16][128];  // A[row][k], B[col][k]
  for (int r = 0; r < 16; ++r)
    for (int k = 0; k < 128; ++k) { A[r][k] = rand() % 16 - 8; B[r][k] = rand() % 16 - 8; }
  int bad_total = 0;
  for (int fmt = 2; fmt <= 3; ++fmt) {
    uint32_t ha[64 * 6], hb[64 * 6];
    for (int l = 0; l < 64; ++l) {  // assumed map: lane l holds row l & 15, k = 32 (l >> 4) + j
      uint32_t ca[32], cb[32];
      for (int j = 0; j < 32; ++j) {
        const int k = 32 * (l >> 4) + j;
        ca[j] = fmt == 3 ? code_e3m2(A[l & 15][k]) : code_e2m3(A[l & 15][k]);
        cb[j] = fmt == 3 ? code_e3m2(B[l & 15][k]) : code_e2m3(B[l & 15][k]);
      }
      pack32(ca, ha + l * 6);
      pack32(cb, hb + l * 6);
    }
    uint32_t *da, *db; float* dc;
    CK(hipMalloc(&da, sizeof ha)); CK(hipMalloc(&db, sizeof hb)); CK(hipMalloc(&dc, 256 * 4));
    CK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice));
    const int scale = fmt == 3 ? 0x7f7f7f7f : 0x80808080;
    if (fmt == 3) hipLaunchKernelGGL(one_mfma<3>, dim3(1), dim3(64), 0, 0, da, db, dc, scale, 1);
    else hipLaunchKernelGGL(one_mfma<2>, dim3(1), dim3(64), 0, 0, da, db, dc, scale, 1);
    CK(hipDeviceSynchronize());
    float hc[256];
    CK(hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost));
    // C map (16x16, shape-determined): lane l, reg i -> row 4 (l >> 4) + i, col l & 15. The
    // intrinsic's first operand is the MFMA's A (rows), the second B (cols).
    int bad = 0, bad_t = 0;
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i) {
        const int row = 4 * (l >> 4) + i, col = l & 15;
        long ref = 0, reft = 0;
        for (int k = 0; k < 128; ++k) { ref += (long)A[row][k] * B[col][k]; reft += (long)A[col][k] * B[row][k]; }
        if ((double)hc[l * 4 + i] != (double)ref) ++bad;
        if ((double)hc[l * 4 + i] != (double)reft) ++bad_t;
      }
    printf("fmt %d one MFMA: mismatches %d / 256 (transposed map: %d); c[0] = %.1f\n", fmt, bad, bad_t, hc[0]);
    bad_total += bad < bad_t ? bad : bad_t;
    // worst case chain: all -8, K = 14336 (112 MFMAs)
    for (int l = 0; l < 64; ++l) {
      uint32_t cm[32];
      for (int j = 0; j < 32; ++j) cm[j] = fmt == 3 ? code_e3m2(-8) : code_e2m3(-8);
      pack32(cm, ha + l * 6);
    }
    CK(hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice));
    if (fmt == 3) hipLaunchKernelGGL(one_mfma<3>, dim3(1), dim3(64), 0, 0, da, da, dc, scale, 112);
    else hipLaunchKernelGGL(one_mfma<2>, dim3(1), dim3(64), 0, 0, da, da, dc, scale, 112);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost));
    int bad2 = 0;
    for (int i = 0; i < 256; ++i) bad2 += hc[i] != 917504.0f;
    printf("fmt %d K=14336 (-8)x(-8) chain: c = %.1f, mismatches %d / 256 (expect 917504)\n", fmt, hc[0], bad2);
    bad_total += bad2;
    // mixed-sign chain: alternate rows of +7 / -8 so partial sums swing; K = 14336
    CK(hipFree(da)); CK(hipFree(db)); CK(hipFree(dc));
  }
  // ---- issue rate ----
  float* sink;
  CK(hipMalloc(&sink, 512 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[3] = {"fp6 e3m2 16x16x128", "i8 16x16x64", "fp4 16x16x128"};
  const double macs[3] = {16.0 * 16 * 128, 16.0 * 16 * 64, 16.0 * 16 * 128};
  for (int kind = 0; kind < 3; ++kind) {
    const int iters = 1024, grid = 1024;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (kind == 0) hipLaunchKernelGGL(rate<0>, dim3(grid), dim3(512), 0, 0, sink, iters);
      else if (kind == 1) hipLaunchKernelGGL(rate<1>, dim3(grid), dim3(512), 0, 0, sink, iters);
      else hipLaunchKernelGGL(rate<2>, dim3(grid), dim3(512), 0, 0, sink, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double ops = 2.0 * macs[kind] * 4 * iters * 8 * grid;
      if (rep) printf("rate %-20s %.3f ms  %.0f T(FL)OP/s\n", names[kind], ms, ops / ms / 1e9);
    }
  }
  printf(bad_total ? "PROBE FAIL\n" : "PROBE OK\n");
  return 0;
}
