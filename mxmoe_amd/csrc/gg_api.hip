// gg_api.hip — host side of libmxmoe_gg.so: the C-ABI declared in include/mxmoe_gg.h.
//
// Reference behaviour replaced (SeaCatComplexes/MxMoE):
//   host API groupgemm_hz_fused_<i> ........ kernel_sketch.py:82-145 (prefix sum on host,
//                                             cudaMalloc/Memcpy/Free per call, grid = #SMs)
//   registry FuncType / kernel selection ... registry.cuh:28-107, compose_kernel.py:482-529
//   qtype dispatch + "quant type not supported" ... compose_kernel.py:47-57, 421-479
// Here: the planner writes a 64-B-per-problem table into a caller-owned workspace once, the
// launch is allocation- and sync-free (hipGraph capturable), errors are status codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mxmoe_gg.h"
#include "gg_device.h"

using namespace mxmoe;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(MXMOE_GG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct TileGeom {
  int bm, bn, bkb, threads;
};

struct Variant {
  const char* name;
  TileGeom geom[QT_COUNT];  // indexed by QType
  int threads;
  int lds_bytes;
  void (*launch)(const GGArgs&, int grid, hipStream_t);
};

template <class C16, class C8, class C4>
void launch_fused(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_fused_kernel<C16, C8, C4>), dim3(grid), dim3(C16::kThreads), 0, s, a);
}

template <class C16, class C8, class C4>
Variant make_variant(const char* name) {
  Variant v;
  v.name = name;
  v.geom[QT_F16] = {C16::BM, C16::BN, C16::BKB, C16::kThreads};
  v.geom[QT_I8] = {C8::BM, C8::BN, C8::BKB, C8::kThreads};
  v.geom[QT_I4] = {C4::BM, C4::BN, C4::BKB, C4::kThreads};
  v.threads = C16::kThreads;
  v.lds_bytes = FusedCfg<C16, C8, C4>::LDS_BYTES;
  v.launch = &launch_fused<C16, C8, C4>;
  return v;
}

typedef TileCfg<128, 128, 2, 2, 2> T128x128;
typedef TileCfg<256, 128, 2, 2, 1> T256x128;
typedef TileCfg<128, 256, 2, 2, 1> T128x256;

const std::vector<Variant>& variants() {
  static const std::vector<Variant> v = {
      make_variant<T128x128, T128x128, T128x128>("fused_128x128_w4"),
      make_variant<T256x128, T256x128, T256x128>("fused_256x128_w4"),
      make_variant<T128x256, T128x256, T128x256>("fused_128x256_w4"),
  };
  return v;
}

constexpr int kDefaultVariant = 0;

int qtype_of(int a_bits, int w_bits, int gsize, int sym, int* qt) {
  if (a_bits == 16 && w_bits == 16) {
    *qt = QT_F16;
    return MXMOE_GG_OK;
  }
  if (a_bits == 8 && w_bits == 8 && gsize == -1 && sym) {
    *qt = QT_I8;
    return MXMOE_GG_OK;
  }
  if (a_bits == 4 && w_bits == 4 && gsize == -1 && sym) {
    *qt = QT_I4;
    return MXMOE_GG_OK;
  }
  return fail(MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported: w%da%d_g%d_%s", w_bits, a_bits, gsize,
              sym ? "sym" : "asym");
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Workspace: [GGMeta x P][ptr_A x P][ptr_B x P][ptr_SA x P][ptr_SB x P][ptr_C x P], 256-B aligned.
size_t ws_meta_bytes(int P) { return align_up((size_t)P * sizeof(GGMeta), 256); }
size_t ws_ptr_bytes(int P) { return align_up((size_t)P * sizeof(void*), 256); }
size_t ws_total_bytes(int P) { return ws_meta_bytes(P) + 5 * ws_ptr_bytes(P); }

struct HostProblem {
  const void *A, *B, *SA, *SB;
  void* C;
  int M, N, K, a_bits, w_bits, gsize, sym;
  int64_t lda, ldb, ldc;  // 16-bit words, 0 = dense
};

// Validate one problem and fill its table row (tile_begin filled by the caller).
int build_meta(const HostProblem& p, int idx, const Variant& v, bool check_ptrs, GGMeta* m) {
  if (p.M < 0 || p.N < 0 || p.K < 0) return fail(MXMOE_GG_ERR_INVALID, "problem %d: negative shape", idx);
  int qt = 0;
  int st = qtype_of(p.a_bits, p.w_bits, p.gsize, p.sym, &qt);
  if (st) return fail(st, "problem %d: %s", idx, g_last_error.c_str());
  const int abits = qt == QT_F16 ? 16 : p.a_bits;
  const int64_t kbits = (int64_t)p.K * abits;
  if (kbits % 128 != 0)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: K=%d must be a multiple of %d for %d-bit data (16-B rows)", idx,
                p.K, (int)(128 / abits), abits);
  if (qt != QT_F16 && p.K > 131072)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: K=%d exceeds the exact int32 accumulation bound 131072", idx, p.K);
  if (p.N % 8 != 0) return fail(MXMOE_GG_ERR_INVALID, "problem %d: N=%d must be a multiple of 8", idx, p.N);
  const int64_t kbytes = kbits / 8;
  const int64_t lda_b = p.lda ? p.lda * 2 : kbytes;
  const int64_t ldb_b = p.ldb ? p.ldb * 2 : kbytes;
  const int64_t ldc = p.ldc ? p.ldc : p.N;
  if (lda_b < kbytes || ldb_b < kbytes || (lda_b % 16) || (ldb_b % 16))
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: lda/ldb must be >= K row and a multiple of 8 words", idx);
  if (ldc < p.N || (ldc % 8)) return fail(MXMOE_GG_ERR_INVALID, "problem %d: ldc must be >= N and a multiple of 8", idx);
  if (check_ptrs && p.M > 0 && p.N > 0) {  // empty problems are dropped by the planner
    if (!p.A || !p.B || !p.C) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL A/B/C", idx);
    if (qt != QT_F16 && (!p.SA || !p.SB)) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL scale pointer", idx);
    if (((uintptr_t)p.A | (uintptr_t)p.B | (uintptr_t)p.C) & 15)
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: A/B/C must be 16-byte aligned", idx);
    if (qt != QT_F16 && (((uintptr_t)p.SA | (uintptr_t)p.SB) & 1))
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: scales must be 2-byte aligned", idx);
  }
  const TileGeom& g = v.geom[qt];
  memset(m, 0, sizeof(*m));
  m->M = p.M;
  m->N = p.N;
  m->K = p.K;
  m->qtype = qt;
  m->tiles_n = (p.N + g.bn - 1) / g.bn;
  m->kbytes = (int32_t)kbytes;
  m->lda_b = lda_b;
  m->ldb_b = ldb_b;
  m->ldc = ldc;
  return MXMOE_GG_OK;
}

// Plan problems into host buffers. Order: problems with more K bytes per tile (= longer tiles)
// first, so the longest workgroups are dispatched first and the tail is short (LPT-style).
int plan_host(const std::vector<HostProblem>& probs, int variant, bool check_ptrs, std::vector<GGMeta>& meta,
              std::vector<int>& order, int* total_tiles) {
  const Variant& v = variants()[variant];
  const int P = (int)probs.size();
  std::vector<GGMeta> all(P);
  std::vector<int64_t> tiles(P, 0);
  for (int i = 0; i < P; ++i) {
    int st = build_meta(probs[i], i, v, check_ptrs, &all[i]);
    if (st) return st;
    const TileGeom& g = v.geom[all[i].qtype];
    if (probs[i].M > 0 && probs[i].N > 0) tiles[i] = (int64_t)((probs[i].M + g.bm - 1) / g.bm) * all[i].tiles_n;
  }
  order.clear();
  for (int i = 0; i < P; ++i)
    if (tiles[i] > 0) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    // per-tile cost ~ tile area * K bytes (MFMA work per byte is equal for int8/int4 and half for fp16)
    auto cost = [&](int i) {
      const TileGeom& g = v.geom[all[i].qtype];
      const double w = all[i].qtype == QT_F16 ? 2.0 : 1.0;
      return w * (double)g.bm * g.bn * (all[i].qtype == QT_I4 ? 2.0 * all[i].kbytes : (double)all[i].kbytes);
    };
    return cost(a) > cost(b);
  });
  int64_t acc = 0;
  meta.clear();
  for (int i : order) {
    GGMeta m = all[i];
    m.tile_begin = (int32_t)acc;
    acc += tiles[i];
    meta.push_back(m);
  }
  if (acc > INT32_MAX / 2) return fail(MXMOE_GG_ERR_INVALID, "too many tiles (%lld)", (long long)acc);
  *total_tiles = (int)acc;
  return MXMOE_GG_OK;
}

int check_variant(int variant) {
  if (variant < 0 || variant >= (int)variants().size())
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "variant %d not compiled (have %d)", variant, (int)variants().size());
  return MXMOE_GG_OK;
}

}  // namespace

extern "C" {

int mxmoe_gg_abi_version(void) { return MXMOE_GG_ABI_VERSION; }

const char* mxmoe_gg_last_error(void) { return g_last_error.c_str(); }

int mxmoe_gg_variant_count(void) { return (int)variants().size(); }

int mxmoe_gg_list_variants(char* buf, size_t n) {
  static const char* qnames[QT_COUNT] = {"fp16", "w8a8_g-1_sym", "w4a4_g-1_sym"};
  std::string out;
  const auto& vs = variants();
  for (size_t i = 0; i < vs.size(); ++i) {
    char line[1024];
    int off = snprintf(line, sizeof(line), "%zu %s", i, vs[i].name);
    for (int q = 0; q < QT_COUNT; ++q) {
      const TileGeom& g = vs[i].geom[q];
      const int bits = q == QT_F16 ? 16 : (q == QT_I8 ? 8 : 4);
      off += snprintf(line + off, sizeof(line) - off, " %s=TileConfig(BM=%d, BN=%d, BK=%d, WM=%d, WN=%d, WK=1, STAGE=2)",
                      qnames[q], g.bm, g.bn, g.bkb * 8 / bits, 2, g.threads / 128);
    }
    out += line;
    out += "\n";
  }
  if (buf && n > 0) {
    size_t c = std::min(n - 1, out.size());
    memcpy(buf, out.data(), c);
    buf[c] = 0;
  }
  return (int)vs.size();
}

int mxmoe_gg_variant_tile(int variant, int a_bits, int w_bits, int32_t* bm, int32_t* bn, int32_t* bk_bytes,
                          int32_t* threads) {
  int st = check_variant(variant);
  if (st) return st;
  int qt = 0;
  st = qtype_of(a_bits, w_bits, -1, 1, &qt);
  if (st) return st;
  const TileGeom& g = variants()[variant].geom[qt];
  if (bm) *bm = g.bm;
  if (bn) *bn = g.bn;
  if (bk_bytes) *bk_bytes = g.bkb;
  if (threads) *threads = g.threads;
  return MXMOE_GG_OK;
}

int mxmoe_gg_workspace_size(int problem_count, size_t* bytes) {
  if (problem_count < 0 || !bytes) return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_workspace_size");
  *bytes = ws_total_bytes(std::max(problem_count, 1));
  return MXMOE_GG_OK;
}

int mxmoe_gg_plan(const mxmoe_gg_problem* problems, int problem_count, int variant, void* workspace,
                  size_t workspace_bytes, void* stream, mxmoe_gg_plan_info* info) {
  if (problem_count < 0 || (problem_count > 0 && !problems) || !info)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_plan");
  int st = check_variant(variant);
  if (st) return st;
  std::vector<HostProblem> hp(problem_count);
  for (int i = 0; i < problem_count; ++i) {
    const mxmoe_gg_problem& p = problems[i];
    hp[i] = HostProblem{p.A,      p.B,      p.scale_a, p.scale_b, p.C,   p.M,   p.N,  p.K,
                        p.a_bits, p.w_bits, p.gsize,   p.sym,     p.lda, p.ldb, p.ldc};
  }
  std::vector<GGMeta> meta;
  std::vector<int> order;
  int total = 0;
  st = plan_host(hp, variant, true, meta, order, &total);
  if (st) return st;
  const int P = (int)meta.size();
  const size_t need = ws_total_bytes(std::max(P, 1));
  if (!workspace || workspace_bytes < need)
    return fail(MXMOE_GG_ERR_WORKSPACE, "workspace too small: need %zu bytes, have %zu", need, workspace_bytes);
  // host image of the workspace
  std::vector<uint8_t> img(need, 0);
  memcpy(img.data(), meta.data(), (size_t)P * sizeof(GGMeta));
  const size_t mb = ws_meta_bytes(std::max(P, 1)), pb = ws_ptr_bytes(std::max(P, 1));
  const void** pa = reinterpret_cast<const void**>(img.data() + mb);
  const void** pbb = reinterpret_cast<const void**>(img.data() + mb + pb);
  const void** psa = reinterpret_cast<const void**>(img.data() + mb + 2 * pb);
  const void** psb = reinterpret_cast<const void**>(img.data() + mb + 3 * pb);
  void** pc = reinterpret_cast<void**>(img.data() + mb + 4 * pb);
  for (int j = 0; j < P; ++j) {
    const HostProblem& p = hp[order[j]];
    pa[j] = p.A;
    pbb[j] = p.B;
    psa[j] = p.SA;
    psb[j] = p.SB;
    pc[j] = p.C;
  }
  HIP_TRY(hipMemcpyAsync(workspace, img.data(), need, hipMemcpyHostToDevice, (hipStream_t)stream));
  // the host image is pageable: make sure the runtime has consumed it before it goes away
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  const Variant& v = variants()[variant];
  info->variant = variant;
  info->problem_count = P;
  info->total_tiles = total;
  info->grid = total;
  info->block = v.threads;
  info->lds_bytes = v.lds_bytes;
  info->workspace_bytes = (int64_t)need;
  info->workspace = workspace;
  return MXMOE_GG_OK;
}

int mxmoe_gg_launch(const mxmoe_gg_plan_info* info, void* stream) {
  if (!info) return fail(MXMOE_GG_ERR_INVALID, "NULL plan");
  int st = check_variant(info->variant);
  if (st) return st;
  if (info->total_tiles == 0) return MXMOE_GG_OK;
  const int P = info->problem_count;
  const uint8_t* ws = static_cast<const uint8_t*>(info->workspace);
  const size_t mb = ws_meta_bytes(std::max(P, 1)), pb = ws_ptr_bytes(std::max(P, 1));
  GGArgs a;
  a.meta = reinterpret_cast<const GGMeta*>(ws);
  a.ptr_A = reinterpret_cast<const void* const*>(ws + mb);
  a.ptr_B = reinterpret_cast<const void* const*>(ws + mb + pb);
  a.ptr_SA = reinterpret_cast<const void* const*>(ws + mb + 2 * pb);
  a.ptr_SB = reinterpret_cast<const void* const*>(ws + mb + 3 * pb);
  a.ptr_C = reinterpret_cast<void* const*>(ws + mb + 4 * pb);
  a.P = P;
  a.total_tiles = info->total_tiles;
  variants()[info->variant].launch(a, info->grid, (hipStream_t)stream);
  HIP_TRY(hipGetLastError());
  return MXMOE_GG_OK;
}

int mxmoe_gg_run(const mxmoe_gg_problem* problems, int problem_count, int variant, void* workspace,
                 size_t workspace_bytes, void* stream) {
  mxmoe_gg_plan_info info;
  int st = mxmoe_gg_plan(problems, problem_count, variant, workspace, workspace_bytes, stream, &info);
  if (st) return st;
  return mxmoe_gg_launch(&info, stream);
}

// Reference-compatible entry point (registry.cuh:28-39). The pointer arrays stay on the device
// and are read by the kernel in place; only the planner table is uploaded.
int groupgemm_mxmoe(void** ptr_As, void** ptr_Bs, void** ptr_scale_a, void** ptr_scale_b, void** ptr_Cs,
                    void** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                    mxmoe_dim3* problem_sizes, mxmoe_dim3* h_problem_sizes, mxmoe_qparams* qbits_list,
                    mxmoe_qparams* h_qbits_list, int problem_count) {
  (void)ptr_Ds;
  (void)ldas;
  (void)ldbs;
  (void)ldcs;
  (void)ldds;
  (void)problem_sizes;
  (void)qbits_list;
  if (problem_count < 0 || !h_problem_sizes || !h_qbits_list)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to groupgemm_mxmoe");
  std::vector<HostProblem> hp(problem_count);
  for (int i = 0; i < problem_count; ++i) {
    hp[i] = HostProblem{nullptr,
                        nullptr,
                        nullptr,
                        nullptr,
                        nullptr,
                        (int)h_problem_sizes[i].x,
                        (int)h_problem_sizes[i].y,
                        (int)h_problem_sizes[i].z,
                        h_qbits_list[i].a_bits,
                        h_qbits_list[i].w_bits,
                        h_qbits_list[i].gsize,
                        h_qbits_list[i].sym,
                        0,
                        0,
                        0};
  }
  std::vector<GGMeta> meta;
  std::vector<int> order;
  int total = 0;
  int st = plan_host(hp, kDefaultVariant, false, meta, order, &total);
  if (st) return st;
  if (total == 0) return MXMOE_GG_OK;
  // The kernel indexes pointer arrays by table row, so the caller's arrays can only be used in
  // place when the planner kept the caller's order; otherwise gather them on the device.
  const int P = (int)meta.size();
  const size_t mb = ws_meta_bytes(P), pb = ws_ptr_bytes(P), need = ws_total_bytes(P);
  thread_local void* ws = nullptr;
  thread_local size_t ws_cap = 0;
  if (ws_cap < need) {
    if (ws) HIP_TRY(hipFree(ws));
    ws = nullptr;
    ws_cap = 0;
    HIP_TRY(hipMalloc(&ws, need));
    ws_cap = need;
  }
  // gather the caller's device pointer arrays through the host (same sync cost class as the
  // reference's per-call cudaMemcpy, kernel_sketch.py:102-104)
  std::vector<void*> hA(problem_count), hB(problem_count), hSA(problem_count), hSB(problem_count), hC(problem_count);
  HIP_TRY(hipMemcpy(hA.data(), ptr_As, problem_count * sizeof(void*), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(hB.data(), ptr_Bs, problem_count * sizeof(void*), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(hSA.data(), ptr_scale_a, problem_count * sizeof(void*), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(hSB.data(), ptr_scale_b, problem_count * sizeof(void*), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(hC.data(), ptr_Cs, problem_count * sizeof(void*), hipMemcpyDeviceToHost));
  std::vector<uint8_t> img(need, 0);
  memcpy(img.data(), meta.data(), (size_t)P * sizeof(GGMeta));
  for (int j = 0; j < P; ++j) {
    const int i = order[j];
    reinterpret_cast<void**>(img.data() + mb)[j] = hA[i];
    reinterpret_cast<void**>(img.data() + mb + pb)[j] = hB[i];
    reinterpret_cast<void**>(img.data() + mb + 2 * pb)[j] = hSA[i];
    reinterpret_cast<void**>(img.data() + mb + 3 * pb)[j] = hSB[i];
    reinterpret_cast<void**>(img.data() + mb + 4 * pb)[j] = hC[i];
  }
  HIP_TRY(hipMemcpy(ws, img.data(), need, hipMemcpyHostToDevice));
  const Variant& v = variants()[kDefaultVariant];
  mxmoe_gg_plan_info info;
  info.variant = kDefaultVariant;
  info.problem_count = P;
  info.total_tiles = total;
  info.grid = total;
  info.block = v.threads;
  info.lds_bytes = v.lds_bytes;
  info.workspace_bytes = (int64_t)need;
  info.workspace = ws;
  return mxmoe_gg_launch(&info, nullptr);
}

}  // extern "C"
