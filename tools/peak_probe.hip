// Peak probe ("confirm the peaks on the box with an MFMA and stream
// microbenchmark"). Prints one JSON object:
//   * MFMA throughput with operands in registers (random data, every CU, 8 waves per CU, 8
//     independent accumulators per wave): v_mfma_i32_16x16x64_i8 and v_mfma_f32_16x16x32_f16 —
//     the two instructions the GroupGEMM kernels issue;
//   * the shader clock those loops ran at (s_memtime cycles / s_memrealtime 100-MHz ticks);
//   * HBM read bandwidth (16-B loads over a 4-GiB buffer, grid-stride).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/peak_probe.hip -o tools/bin/peak_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int NACC = 8;

template <bool I8>
__global__ __launch_bounds__(512) void mfma_loop(const uint32_t* __restrict__ seed, int iters, uint64_t* clk,
                                                 int32_t* sink) {
  const int lane = threadIdx.x & 63;
  v4i a = {(int)seed[lane], (int)seed[lane + 64], (int)seed[lane + 128], (int)seed[lane + 192]};
  v4i b = {(int)seed[lane + 256], (int)seed[lane + 320], (int)seed[lane + 384], (int)seed[lane + 448]};
  v4i ai[NACC];
  v4f af[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) {
    ai[k] = v4i{0, 0, 0, 0};
    af[k] = v4f{0, 0, 0, 0};
  }
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      if constexpr (I8) ai[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, ai[k], 0, 0, 0);
      else af[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), af[k], 0, 0, 0);
    }
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int32_t s = 0;
#pragma unroll
  for (int k = 0; k < NACC; ++k) s += I8 ? ai[k].x + ai[k].w : (int32_t)(af[k].x + af[k].w);
  if (s == 0x7fffffff) sink[threadIdx.x] = s;  // keeps the loop live
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = c1 - c0;
    clk[1] = r1 - r0;
  }
}

__global__ __launch_bounds__(256) void hbm_read(const uint4* __restrict__ p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint32_t> h(512);
  uint32_t x = 12345;
  for (auto& v : h) v = (x = x * 1664525u + 1013904223u);
  uint32_t* seed;
  uint64_t* clk;
  int32_t* sink;
  CHECK(hipMalloc(&seed, 512 * 4));
  CHECK(hipMalloc(&clk, 16));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemcpy(seed, h.data(), 512 * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int grid = cus * 4, iters = 20000;  // 4 x 512-thread workgroups per CU over the launch
  double res[2], ghz[2];
  for (int t = 0; t < 2; ++t) {
    auto launch = [&]() {
      if (t == 0) hipLaunchKernelGGL(mfma_loop<true>, dim3(grid), dim3(512), 0, 0, seed, iters, clk, sink);
      else hipLaunchKernelGGL(mfma_loop<false>, dim3(grid), dim3(512), 0, 0, seed, iters, clk, sink);
    };
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double flop_per = t == 0 ? 2.0 * 16 * 16 * 64 : 2.0 * 16 * 16 * 32;
    res[t] = flop_per * NACC * iters * (double)grid * 8 / (ms * 1e-3) / 1e12;
    uint64_t c[2];
    CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
    ghz[t] = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  }
  const size_t bytes = (size_t)4 << 30;
  uint4* buf;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMemset(buf, 0x5a, bytes));
  const size_t n = bytes / 16;
  hipLaunchKernelGGL(hbm_read, dim3(cus * 16), dim3(256), 0, 0, buf, n, (uint32_t*)sink);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(hbm_read, dim3(cus * 16), dim3(256), 0, 0, buf, n, (uint32_t*)sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("{\"cus\": %d, \"int8_mfma_16x16x64_TOPS\": %.1f, \"int8_loop_clock_GHz\": %.3f, "
         "\"f16_mfma_16x16x32_TFLOPS\": %.1f, \"f16_loop_clock_GHz\": %.3f, \"hbm_read_GBs\": %.0f, "
         "\"note\": \"register operands, random data, 8 waves/CU, 8 independent accumulators per wave\"}\n",
         cus, res[0], ghz[0], res[1], ghz[1], bytes / (best * 1e-3) / 1e9);
  return 0;
}
