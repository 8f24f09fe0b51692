// Store-path probe (round 4 design question): how fast does one CU drain a 256 x 256 fp16 output
// tile (128 KiB) with 16-B buffer stores, and do LDS-DMA loads issued by OTHER waves of the same CU
// wait behind those stores? One 512-thread workgroup per CU (160 KiB of LDS each), `reps` tiles per
// workgroup, s_memtime per workgroup. Prints one JSON line per case.
//   layout 0: each store instruction writes 8 rows x 128 B (v2x's LDS-staged epilogue)
//   layout 1: 16 rows x 64 B (direct from MFMA registers after v_permlane16_swap)
//   pol: 0 plain, 16 sc1 (what v2x uses)
//   role 0: all 8 waves store (16 KiB each); role 1: waves 4-7 store the tile (32 KiB each) while
//   waves 0-3 issue 64 KiB of LDS-DMA (16 x 1 KiB pieces each, L2-resident source) right after the
//   barrier; role 2: loads only (the baseline for role 1's load latency)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/store_probe.hip -o tools/bin/store_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

template <int LAYOUT, int POL, int ROLE>
__global__ __launch_bounds__(512) void probe(uint8_t* out, const uint8_t* src, int reps, int64_t ldc_bytes,
                                             uint64_t* t_store, uint64_t* t_load, uint64_t* t_real) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t tile_bytes = 256 * (uint64_t)ldc_bytes;
  v4u v = {(unsigned)tid, (unsigned)blockIdx.x, 0x3c003c00u, 0x12345678u};
  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, 0x7fffffff, 0x00020000);
  uint64_t st_sum = 0, ld_sum = 0;
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < reps; ++r) {
    uint8_t* tile = out + ((uint64_t)blockIdx.x * reps + r) * tile_bytes;
    __syncthreads();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const bool storer = ROLE == 0 || (ROLE == 1 && wave >= 4);
    const bool loader = ROLE != 0 && wave < 4;
    if (loader) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_src, (lds_void_t*)(lds + (wave * 16 + j) * 1024), 16,
                                                 (uint32_t)(((wave * 16 + j) * 64 + lane) * 16), 0, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ld_sum += __builtin_amdgcn_s_memtime() - c0;
    }
    if (storer) {
      // the wave's share of the tile: ROLE 0: 8 waves x 32 rows x 256 cols... laid out as the GEMM
      // epilogue does (wave sub-tile 128 rows x 64 cols); ROLE 1: waves 4-7 each two sub-tiles
      const int nsub = ROLE == 0 ? 1 : 2;
#pragma unroll
      for (int sub = 0; sub < nsub; ++sub) {
        const int w = ROLE == 0 ? wave : (wave - 4) * 2 + sub;  // 0..7: 2 (M) x 4 (N) sub-tiles of 128 x 64
        uint8_t* base = tile + (uint64_t)(w / 4) * 128 * ldc_bytes + (w % 4) * 128;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int it = 0; it < 16; ++it) {
          int row, col;
          if (LAYOUT == 0) {  // 8 rows x 128 B
            row = it * 8 + (lane >> 3);
            col = (lane & 7) * 16;
          } else {  // 16 rows x 64 B (two 16 x 16 fp16 blocks after permlane16_swap)
            row = (it >> 1) * 16 + (lane & 15);
            col = (it & 1) * 64 + ((lane >> 4) & 1) * 32 + (lane >> 5) * 16;
          }
          v.x += it;
          __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(row * ldc_bytes + col), 0, POL);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sum += __builtin_amdgcn_s_memtime() - c0;
    }
  }
  __syncthreads();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    if (wave == (ROLE == 1 ? 4 : 0)) t_store[blockIdx.x] = st_sum / reps;
    if (wave == 0 && ROLE != 0) t_load[blockIdx.x] = ld_sum / reps;
    if (wave == 0) t_real[blockIdx.x] = r1 - r0;
  }
}

template <int LAYOUT, int POL, int ROLE>
int run(int nwg, int reps, int64_t ldc_bytes, uint8_t* out, const uint8_t* src) {
  uint64_t *ts, *tl, *tr;
  CHECK(hipMalloc(&ts, nwg * 8));
  CHECK(hipMalloc(&tl, nwg * 8));
  CHECK(hipMalloc(&tr, nwg * 8));
  CHECK(hipMemset(ts, 0, nwg * 8));
  CHECK(hipMemset(tl, 0, nwg * 8));
  for (int w = 0; w < 3; ++w) probe<LAYOUT, POL, ROLE><<<nwg, 512>>>(out, src, reps, ldc_bytes, ts, tl, tr);
  CHECK(hipDeviceSynchronize());
  std::vector<uint64_t> hs(nwg), hl(nwg), hr(nwg);
  CHECK(hipMemcpy(hs.data(), ts, nwg * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hl.data(), tl, nwg * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hr.data(), tr, nwg * 8, hipMemcpyDeviceToHost));
  std::sort(hs.begin(), hs.end());
  std::sort(hl.begin(), hl.end());
  std::sort(hr.begin(), hr.end());
  const double st = (double)hs[nwg / 2], ld = (double)hl[nwg / 2];
  printf("{\"layout\": %d, \"pol\": %d, \"role\": %d, \"wgs\": %d, \"ldc_B\": %lld, \"store_cyc_per_tile\": %.0f, "
         "\"store_B_per_cyc\": %.1f, \"load_cyc\": %.0f, \"wall_us_per_tile\": %.3f}\n",
         LAYOUT, POL, ROLE, nwg, (long long)ldc_bytes, st, st > 0 ? 131072.0 / st : 0.0, ld,
         hr[nwg / 2] * 0.01 / reps);
  CHECK(hipFree(ts));
  CHECK(hipFree(tl));
  CHECK(hipFree(tr));
  return 0;
}

int main() {
  const int reps = 16;
  const int64_t ldc_max = 22528;  // qwen2_moe gate_up C row (11264 fp16)
  uint8_t *out, *src;
  CHECK(hipMalloc(&out, (size_t)256 * reps * 256 * ldc_max));
  CHECK(hipMalloc(&src, 1 << 20));
  CHECK(hipMemset(src, 1, 1 << 20));
  for (int64_t ldc : {(int64_t)22528, (int64_t)5632}) {
    for (int nwg : {256, 32}) {
      if (run<0, 16, 0>(nwg, reps, ldc, out, src)) return 1;
      if (run<0, 0, 0>(nwg, reps, ldc, out, src)) return 1;
      if (run<1, 16, 0>(nwg, reps, ldc, out, src)) return 1;
      if (run<1, 0, 0>(nwg, reps, ldc, out, src)) return 1;
      if (run<0, 16, 1>(nwg, reps, ldc, out, src)) return 1;
      if (run<1, 16, 1>(nwg, reps, ldc, out, src)) return 1;
      if (run<0, 16, 2>(nwg, reps, ldc, out, src)) return 1;
    }
  }
  return 0;
}
