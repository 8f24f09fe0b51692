// gg_api.hip — host side of libmxmoe_gg.so: the C-ABI declared in include/mxmoe_gg.h.
//
// Reference behaviour replaced (SeaCatComplexes/MxMoE):
//   host API groupgemm_hz_fused_<i> ........ kernel_sketch.py:82-145 (prefix sum on host,
//                                             cudaMalloc/Memcpy/Free per call, grid = #SMs)
//   tile -> (problem, m, n) by prefix scan .. tile_scheduler.cuh:25-50
//   registry FuncType / kernel selection ... registry.cuh:28-107, compose_kernel.py:482-529
//   qtype dispatch + "quant type not supported" ... compose_kernel.py:47-57, 421-479
// Here: the planner builds an explicit tile table once into a caller-owned workspace — tiles of
// the longest problems first (LPT), grouped into chunks of neighbouring tiles that run together on
// one XCD (shared A rows / B columns hit that XCD's L2) — and the launch is allocation- and
// sync-free (hipGraph capturable). Errors are status codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mxmoe_gg.h"
#include "gg_device.h"
#ifdef MXMOE_LAB
#include "gg_f6.h"   // lab-only fp6 w4a4 route: measured slower than the int4 path
#include "gg_v2q.h"  // lab-only persistent kernel: not compiled into the product library
#include "gg_v4.h"   // lab-only one-wave-per-SIMD 256 x 256 tile
// lab-only operand format: w4a4_g-1_sym with A / B as fp6 images (mxmoe_gg_pack_f6, gg_f6.h)
#define MXMOE_GG_FMT_F6 3
#define MXMOE_GG_F6_ROW_BYTES(K) ((((int64_t)(K) + 127) / 128) * 96)
#endif

using namespace mxmoe;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[768];
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

// Planner A/B switches (MXMOE_GG_BAND, _REGION, _REGION_ROT, _ALIGN, _TAIL_CHUNK, _XCD_RR) are
// read only by the tools-only lab build (-DMXMOE_LAB, libmxmoe_gg_lab.so): the product library's
// tile placement never depends on the caller's environment.
const char* planner_knob(const char* name) {
#ifdef MXMOE_LAB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

struct TileGeom {
  int bm, bn, bkb, threads;
};

enum class Kind { V0, V2, V3 };  // (the fp6 kernel is planned as V3: no split-K, no XCD regions)

struct Variant {
  const char* name;
  Kind kind;
  TileGeom geom[QT_COUNT];  // indexed by QType (main tile)
  int threads;
  int lds_bytes;
  int chunk;           // tiles per XCD chunk (workgroups that run together on one XCD)
  int k_stage_bytes;   // K bytes per row must be a multiple of this (0 = any multiple of 16)
  int tail_bm;         // v2: height of the tail-tile class (0 = none)
  int tail2_bm = 0;    // v2: height of the small-remainder class (0 = none)
  bool persistent = false;  // v2p / v2q: a workgroup walks a planned tile list
  bool silu_epi = false;    // the fp16 / w8a8 / w4a4 tile bodies carry the fused SiLU epilogue
  bool silu_wo = false;     // ... and its weight-only tiles (wo2: the WO_SILU builds)
  int persist_len = 0;      // v2q: 0 = one list per CU (static); L > 0 = lists of L consecutive XCD-queue
                            // tiles, one per block, the hardware dispatching blocks as CUs free up
  int (*lds_of)(int qmask) = nullptr;  // LDS of the build a quant-type set launches (default lds_bytes)
  void (*launch)(const GGArgs&, int grid, int qmask, hipStream_t);  // qmask: 1 << QType present
};

template <class C16, class C8, class C4>
void launch_v0(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  hipLaunchKernelGGL((gg_fused_kernel<C16, C8, C4>), dim3(grid), dim3(C16::kThreads), 0, s, a);
}

template <int ABL, int QM>
void launch_v2_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_v2_kernel<ABL, QM>), dim3(grid), dim3(512), 0, s, a);
}
template <int ABL>
void launch_v2(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  if constexpr ((ABL & kAblMask) != 0) {
    launch_v2_q<ABL, 7>(a, grid, s);
  } else if constexpr ((ABL & kWoAblMask) != 0) {
    launch_v2_q<ABL, 8>(a, grid, s);  // weight-only ablations: w4a16 tiles only
  } else {
#if defined(MXMOE_LAB) && defined(MXMOE_LAB_FAST)
    switch (qmask & 511) {
      case 1: launch_v2_q<ABL, 1>(a, grid, s); break;
      case 2: launch_v2_q<ABL, 2>(a, grid, s); break;
      case 8: launch_v2_q<ABL, 8>(a, grid, s); break;
      default:
        fprintf(stderr, "libmxmoe_gg_lab (fast): quant-type mix %#x not compiled\n", qmask);
        abort();
    }
#elif defined(MXMOE_LAB)
    // lab build: fp16, w8a8, w4a4, w8a8 + w4a4 (LP-1 mixed), w4a16, bf16 only (fast builds)
    switch (qmask & 511) {
      case 1: launch_v2_q<ABL, 1>(a, grid, s); break;
      case 2: launch_v2_q<ABL, 2>(a, grid, s); break;
      case 4: launch_v2_q<ABL, 4>(a, grid, s); break;
      case 6: launch_v2_q<ABL, 6>(a, grid, s); break;
      case 8: launch_v2_q<ABL, 8>(a, grid, s); break;
      case 128: launch_v2_q<ABL, 128>(a, grid, s); break;
      case 256: launch_v2_q<ABL, 256>(a, grid, s); break;
      default:
        fprintf(stderr, "libmxmoe_gg_lab: quant-type mix %#x not compiled in the lab build\n", qmask);
        abort();
    }
#else
    switch (qmask & 511) {
      case 1: launch_v2_q<ABL, 1>(a, grid, s); break;
      case 2: launch_v2_q<ABL, 2>(a, grid, s); break;
      case 4: launch_v2_q<ABL, 4>(a, grid, s); break;
      case 6: launch_v2_q<ABL, 6>(a, grid, s); break;
      case 7: launch_v2_q<ABL, 7>(a, grid, s); break;
      case 8: launch_v2_q<ABL, 8>(a, grid, s); break;    // w4a16 only
      case 10: launch_v2_q<ABL, 10>(a, grid, s); break;  // w4a16 + w8a8 (the reference's hz_fused pairing)
      case 16: launch_v2_q<ABL, 16>(a, grid, s); break;  // w8a16 only
      case 32: launch_v2_q<ABL, 32>(a, grid, s); break;  // w4a4 g128 only
      case 64: launch_v2_q<ABL, 64>(a, grid, s); break;  // w2a16 only
      case 128: launch_v2_q<ABL, 128>(a, grid, s); break;  // w8a8 E4M3 only
      case 256: launch_v2_q<ABL, 256>(a, grid, s); break;  // bf16 only
      // any other mix: every tile body in one kernel. The staggered int bodies leave no register
      // room for that (the compiler spilled inside their K loops), so the fallback is plain v2;
      // the 2-bit weight-only body only joins it when the mix has one (it costs 12 B of prologue
      // spill there, tests/test_codegen.py)
      default:
        if (qmask & ((1 << QT_F8) | (1 << QT_BF16))) launch_v2_q<0, 511>(a, grid, s);
        else if (qmask & (1 << QT_W2A16)) launch_v2_q<0, 127>(a, grid, s);
        else launch_v2_q<0, 63>(a, grid, s);
        break;
    }
#endif
  }
}

// v3 is specialised on the set of quant types the plan contains (mask 1 << QType)
template <int BN, int WN, int NBUF, int DIST, int QM, int OPT>
void launch_v3_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_v3_kernel<BN, WN, NBUF, DIST, QM, OPT>), dim3(grid), dim3(V3Cfg<256, BN, WN>::NT), 0, s, a);
}
template <int BN, int WN, int NBUF, int DIST, int OPT = 0>
void launch_v3(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  switch (qmask & 7) {
    case 1: launch_v3_q<BN, WN, NBUF, DIST, 1, OPT>(a, grid, s); break;
    case 2: launch_v3_q<BN, WN, NBUF, DIST, 2, OPT>(a, grid, s); break;
    case 4: launch_v3_q<BN, WN, NBUF, DIST, 4, OPT>(a, grid, s); break;
    case 6: launch_v3_q<BN, WN, NBUF, DIST, 6, OPT>(a, grid, s); break;
    default: launch_v3_q<BN, WN, NBUF, DIST, 7, OPT>(a, grid, s); break;
  }
}

template <int QM, int TRACE>
void launch_v2p_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_v2p_kernel<QM, TRACE>), dim3(grid), dim3(512), 0, s, a);
}
template <int TRACE = 0>
void launch_v2p(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  switch (qmask & 511) {
    case 1: launch_v2p_q<1, TRACE>(a, grid, s); break;
    case 2: launch_v2p_q<2, TRACE>(a, grid, s); break;
    case 256: launch_v2p_q<256, TRACE>(a, grid, s); break;
    default: launch_v2p_q<511, TRACE>(a, grid, s); break;  // every tile body
  }
}

#ifdef MXMOE_LAB
template <int QM, int TRACE, int SAUX, int FILLALL>
void launch_v2q_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_v2q_kernel<QM, TRACE, SAUX, FILLALL>), dim3(grid), dim3(512), 0, s, a);
}
template <int TRACE = 0, int SAUX = 16, int FILLALL = 0>
void launch_v2q(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  switch (qmask & 511) {
    case 1: launch_v2q_q<1, TRACE, SAUX, FILLALL>(a, grid, s); break;
    case 2: launch_v2q_q<2, TRACE, SAUX, FILLALL>(a, grid, s); break;
#ifndef MXMOE_LAB_FAST
    case 4: launch_v2q_q<4, TRACE, SAUX, FILLALL>(a, grid, s); break;
    case 6: launch_v2q_q<6, TRACE, SAUX, FILLALL>(a, grid, s); break;
    case 256: launch_v2q_q<256, TRACE, SAUX, FILLALL>(a, grid, s); break;
    default: launch_v2q_q<511, TRACE, SAUX, FILLALL>(a, grid, s); break;  // every tile body
#else
    default:
      fprintf(stderr, "libmxmoe_gg_lab (fast): v2q quant-type mix %#x not compiled\n", qmask);
      abort();
#endif
  }
}

#endif  // MXMOE_LAB

template <int ABL, int QM, int NWG>
void launch_wo2_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_wo2_kernel<ABL, QM, NWG>), dim3(grid), dim3(512), 0, s, a);
}
// quant-type sets launched at the variant's NWG (the rest, with 8-bit weight-only problems, run the
// 2-WG/CU build): keep in step with the switch below
constexpr bool wo2_full_nwg(int qm) { return qm == 8 || qm == 64 || qm == 10 || qm == 1 || qm == 2 || qm == 4 || qm == 6; }
// plan-info qtype_mask bit: a weight-only problem carries MXMOE_GG_EPI_SILU_MUL (selects the WO_SILU
// build; with it only the w4a16 and w4a16 + w8a8 sets run at the variant's NWG)
constexpr int kQmaskWoSilu = 1 << 16;
constexpr bool wo2_full_nwg_silu(int qm) { return qm == 8 || qm == 10; }
template <int NWG>
int wo2_launch_lds(int qmask) {
  const bool full = (qmask & kQmaskWoSilu) ? wo2_full_nwg_silu(qmask & 511) : wo2_full_nwg(qmask & 511);
  return full ? wo2_lds_bytes<NWG>() : wo2_lds_bytes<2>();
}
template <int ABL, int NWG>
void launch_wo2(const GGArgs& a, int grid, int qmask, hipStream_t s) {
#ifdef MXMOE_LAB_FAST
  switch (qmask & 511) {  // fast lab build: the w4a16 and w4a16 + w8a8 sets only
    case 8: launch_wo2_q<ABL, 8, NWG>(a, grid, s); break;
    case 10: launch_wo2_q<ABL, 10, NWG>(a, grid, s); break;
    case 16: launch_wo2_q<ABL, 16, NWG>(a, grid, s); break;  // (lab: w8a16 at the variant's NWG)
    default:
      fprintf(stderr, "libmxmoe_gg_lab (fast): wo2 quant-type mix %#x not compiled\n", qmask);
      abort();
  }
#else
  if (qmask & kQmaskWoSilu) {  // weight-only problems with the fused SiLU epilogue (WO_SILU builds)
    constexpr int AS = ABL | WO_SILU;
    switch (qmask & 511) {
      case 8: launch_wo2_q<AS, 8, NWG>(a, grid, s); break;    // w4a16
      case 10: launch_wo2_q<AS, 10, NWG>(a, grid, s); break;  // w4a16 + w8a8 (any other mix: the wide
                                                              // 2-WG/CU builds below)
      case 16: launch_wo2_q<AS, 16, 2>(a, grid, s); break;
      default: launch_wo2_q<AS, 95, 2>(a, grid, s); break;
    }
    return;
  }
  switch (qmask & 511) {
    case 8: launch_wo2_q<ABL, 8, NWG>(a, grid, s); break;    // w4a16 only
    case 64: launch_wo2_q<ABL, 64, NWG>(a, grid, s); break;  // w2a16 only
    case 10: launch_wo2_q<ABL, 10, NWG>(a, grid, s); break;  // w4a16 + w8a8 (hz_fused pairing)
    case 1: launch_wo2_q<ABL, 1, NWG>(a, grid, s); break;    // fp16 only
    case 2: launch_wo2_q<ABL, 2, NWG>(a, grid, s); break;    // w8a8 only
    case 4: launch_wo2_q<ABL, 4, NWG>(a, grid, s); break;    // w4a4 only
    case 6: launch_wo2_q<ABL, 6, NWG>(a, grid, s); break;    // w4a4 + w8a8 (LP-1 mixed)
    // the 8-bit body does not fit 80 VGPRs (3 workgroups per CU) without spilling: calls with w8a16
    // problems run the 2-WG/CU build of the same tiles (same plan: placement only assumes more slots)
    case 16: launch_wo2_q<ABL, 16, 2>(a, grid, s); break;  // w8a16 only
    default: launch_wo2_q<ABL, 95, 2>(a, grid, s); break;  // any mix of fp16, w8a8, w4a4 and weight-only
  }
#endif
}

template <class C16, class C8, class C4>
Variant make_v0(const char* name) {
  Variant v;
  v.name = name;
  v.kind = Kind::V0;
  v.geom[QT_F16] = {C16::BM, C16::BN, C16::BKB, C16::kThreads};
  v.geom[QT_I8] = {C8::BM, C8::BN, C8::BKB, C8::kThreads};
  v.geom[QT_I4] = {C4::BM, C4::BN, C4::BKB, C4::kThreads};
  for (int q : {QT_W4A16, QT_W8A16, QT_I4G, QT_W2A16, QT_F8, QT_BF16, QT_I4F6}) v.geom[q] = {0, 0, 0, 0};  // v2 kernels only
  v.threads = C16::kThreads;
  v.lds_bytes = FusedCfg<C16, C8, C4>::LDS_BYTES;
  v.chunk = FusedCfg<C16, C8, C4>::LDS_BYTES <= 80 * 1024 ? 64 : 32;  // workgroups per XCD at once
  v.k_stage_bytes = 0;
  v.tail_bm = 0;
  v.launch = &launch_v0<C16, C8, C4>;
  return v;
}

template <int BN, int WN, int NBUF, int DIST, int OPT = 0>
Variant make_v3(const char* name) {
  typedef V3Cfg<256, BN, WN, NBUF, DIST> CT;
  Variant v;
  v.name = name;
  v.kind = Kind::V3;
  for (int q = 0; q < QT_COUNT; ++q) v.geom[q] = {256, BN, 64, CT::NT};  // (weight-only / g128 / fp8 / bf16 cleared below)
  for (int q : {QT_W4A16, QT_W8A16, QT_I4G, QT_W2A16, QT_F8, QT_BF16, QT_I4F6}) v.geom[q] = {0, 0, 0, 0};  // v2 kernels only
  v.threads = CT::NT;
  v.lds_bytes = CT::LDS_BYTES;
  v.chunk = 32 * (160 * 1024 / CT::LDS_BYTES >= 2 ? 2 : 1);  // workgroups per XCD at once
  v.k_stage_bytes = 0;
  v.tail_bm = 128;
  v.launch = &launch_v3<BN, WN, NBUF, DIST, OPT>;
  v.silu_epi = true;  // epilogue_v3
  return v;
}

#ifdef MXMOE_LAB
template <int NBUF, int DIST, int OPT>
void launch_f6(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  (void)qmask;  // QT_I4F6 only
  hipLaunchKernelGGL((gg_f6_kernel<NBUF, DIST, OPT>), dim3(grid), dim3(512), 0, s, a);
}

// fp6 w4a4 tiles (gg_f6.h): 256 x 256 (+ 128-row tail class), one 512-thread workgroup per CU
template <int NBUF, int DIST, int OPT = 0>
Variant make_f6(const char* name) {
  typedef F6Cfg<256, 256, 2, 4, NBUF, DIST> CT;
  Variant v;
  v.name = name;
  v.kind = Kind::V3;
  for (int q = 0; q < QT_COUNT; ++q) v.geom[q] = {0, 0, 0, 0};
  v.geom[QT_I4F6] = {256, 256, CT::SKB, CT::NT};
  v.threads = CT::NT;
  v.lds_bytes = CT::LDS_BYTES;
  v.chunk = 32;
  v.k_stage_bytes = 0;  // (image rows are whole stages by construction)
  v.tail_bm = 128;
  v.launch = &launch_f6<NBUF, DIST, OPT>;
  return v;
}
#endif  // MXMOE_LAB

// the v2 family's geometry (launch set by the caller)
Variant v2_base(const char* name, int lds_bytes) {
  Variant v;
  v.name = name;
  v.kind = Kind::V2;
  for (int q = 0; q < QT_COUNT; ++q) v.geom[q] = {256, 256, 128, 512};
  v.geom[QT_W4A16] = {256, 256, 32, 512};  // 64-K stages: 32 B of 4-bit codes per row
  v.geom[QT_W8A16] = {256, 256, 64, 512};
  v.geom[QT_W2A16] = {256, 256, 16, 512};  // 64-K stages: 16 B of 2-bit codes per row
  v.geom[QT_I4G] = {256, 256, 128, 512};  // w4a4 g128 (gg_tile_g128): 256 / 128-row classes as int4
  v.geom[QT_I4F6] = {0, 0, 0, 0};         // fp6 images: the f6 kernel only
  v.threads = 512;
  v.lds_bytes = lds_bytes;
  v.chunk = 32;  // one 512-thread workgroup per CU, 32 CUs per XCD
  v.k_stage_bytes = 0;  // K tails handled in-kernel (last stage)
  v.tail_bm = 128;
  v.tail2_bm = 64;  // <= 64 remaining rows, fp16 / weight-only problems (small batches)
  return v;
}

template <int ABL = 0>
Variant make_v2(const char* name) {
  Variant v = v2_base(name, (ABL & V2_B3) ? 160 * 1024 : V2Cfg<256>::LDS_BYTES + V2_LDS_EXTRA);
  v.launch = &launch_v2<ABL>;
  v.silu_epi = true;  // gg_tile_v2's epilogue
  return v;
}


bool is_weightonly(int qt);

// wo2: weight-only problems only, 64-row tiles, NWG workgroups per CU (gg_wo2_kernel)
template <int ABL = 0, int NWG = 2>
Variant make_wo2(const char* name) {
  Variant v = v2_base(name, wo2_lds_bytes<NWG>());  // (no v2 kernel instantiated for the wo flags)
  for (int q = 0; q < QT_COUNT; ++q)
    if (!is_weightonly(q)) v.geom[q] = {0, 0, 0, 0};
    else v.geom[q].bm = 64;
  v.geom[QT_I8] = {64, 128, 128, 512};  // w8a8 (beside weight-only problems): 64 x 128 int8 tiles
  v.geom[QT_F16] = {64, 128, 128, 512};  // fp16: 64 x 128 tiles (64-K stages)
  v.geom[QT_I4] = {64, 128, 128, 512};   // w4a4: 64 x 128 tiles (256-K stages)
  v.lds_bytes = wo2_lds_bytes<NWG>();
  v.chunk = 32 * NWG;  // NWG workgroups per CU, 32 CUs per XCD
  v.tail_bm = 0;
  v.tail2_bm = 0;
  v.launch = &launch_wo2<ABL, NWG>;
  v.lds_of = &wo2_launch_lds<NWG>;
  v.silu_epi = true;  // its fp16 / w8a8 / w4a4 problems run gg_tile_v2 64 x 128 bodies (their epilogue)
#ifndef MXMOE_LAB_FAST
  v.silu_wo = true;   // weight-only problems: the WO_SILU builds (launch_wo2)
#endif
  return v;
}

template <int TRACE = 0>
Variant make_v2p(const char* name) {
  Variant v = make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (4 << V2_SPREAD_SHIFT)>(name);
  v.persistent = true;
  v.lds_bytes = 160 * 1024;
  v.launch = &launch_v2p<TRACE>;
  return v;
}

#ifdef MXMOE_LAB
// v2q: the persistent v2x with the register epilogue and the next tile's ring fill before it
// (gg_v2q.h); planned like v2p (per-workgroup tile lists)
template <int TRACE = 0, int SAUX = 16, int FILLALL = 0>
Variant make_v2q(const char* name, int persist_len = 0) {
  Variant v = make_v2p<0>(name);
  v.launch = &launch_v2q<TRACE, SAUX, FILLALL>;
  v.persist_len = persist_len;
  return v;
}
// v4d (gg_v4.h): 256 x 256 tiles (+ 128 / 64-row classes), 4 waves at one per SIMD, fp16 / w8a8 only
template <int QM, int OPT>
void launch_v4_q(const GGArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((gg_v4_kernel<QM, OPT>), dim3(grid), dim3(256), 0, s, a);
}
template <int OPT = 0>
void launch_v4(const GGArgs& a, int grid, int qmask, hipStream_t s) {
  switch (qmask & 511) {
    case 1: launch_v4_q<1, OPT>(a, grid, s); break;
    case 2: launch_v4_q<2, OPT>(a, grid, s); break;
    case 4: launch_v4_q<4, OPT>(a, grid, s); break;
#ifndef MXMOE_LAB_FAST
    case 6: launch_v4_q<6, OPT>(a, grid, s); break;
    default: launch_v4_q<7, OPT>(a, grid, s); break;
#else
    default: launch_v4_q<3, OPT>(a, grid, s); break;
#endif
  }
}
template <int OPT = 0>
Variant make_v4(const char* name) {
  Variant v = v2_base(name, V4Cfg<256>::LDS_BYTES);
  for (int q = 0; q < QT_COUNT; ++q)
    if (q != QT_F16 && q != QT_I8 && q != QT_I4) v.geom[q] = {0, 0, 0, 0};
  v.geom[QT_F16].threads = v.geom[QT_I8].threads = v.geom[QT_I4].threads = 256;
  v.threads = 256;
  v.launch = &launch_v4<OPT>;
  return v;
}
#endif  // MXMOE_LAB

// the small-batch weight-only tile's loop options (gg_tile_wo)
constexpr int kWo3 = WO_SCLATE | WO_ANDOR | WO_MSKIP | WO_SPLIT | WO_NIBPOS;

// the round-3 AUTO default's mainloop flags (variant v2x_256x256_w8_b3_buf_spread_edma, without the
// weight-only options)
constexpr int kV2x = V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (4 << V2_SPREAD_SHIFT);

typedef TileCfg<128, 128, 2, 2, 2> T128x128;
typedef TileCfg<256, 128, 2, 2, 1> T256x128;
typedef TileCfg<128, 256, 2, 2, 1> T128x256;

// the fused SiLU epilogue (MXMOE_GG_EPI_SILU_MUL) lives in the fp16 / w8a8 / w4a4 tile bodies of the
// v2 / v3 kernels (gg_tile_v2, epilogue_v3) — the small-batch wo3 kernel's 64 x 128 bodies of those
// types included (round 6); the persistent, v4d and fp6 lab kernels have none (mxmoe_gg_variant_caps
// reports it). Weight-only problems may carry the flag on wo3 only (Variant::silu_wo, build_meta).
bool has_silu_epilogue(const Variant& v) { return v.silu_epi && !v.persistent; }

// Production variants (libmxmoe_gg.so): every one computes correct results. The lab build
// (-DMXMOE_LAB -> libmxmoe_gg_lab.so, tools only: `python -m mxmoe_amd.build --lab`) compiles the
// v2 family only, with the timing ablations (abl_*, WRONG RESULTS by design) and the mainloop
// experiments, for tools/kbench.py A/B runs (MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so).
const std::vector<Variant>& variants() {
  static const std::vector<Variant> v = {
#ifndef MXMOE_LAB
      // round 4: the product lists what AUTO picks; the round-1/2 kernels (v0
      // register-staged tiles, plain / staggered v2, v3 256 x 256) live on in the lab build
      make_v3<128, 2, 3, 2>("v3_256x128_w4_dma_ring3_2wg"),
      // round 3 (AUTO default): v2s3's LDS image, buffer-form LDS-DMA spread over the first MFMA
      // group of each half stage, issued by waves 0-3 for their SIMD partners too (not on int4
      // tiles) — profiles/r03/lab/
      // (+ the weight-only tiles' pipelined fragment reads and, at 64 rows, the late-wave deferral:
      // +1-4 % on the small-batch w4a16 calls, profiles/r03/wo/)
      // round 5: int4 fragment reads kept unpaired (V2_I4NOPAIR: ds_read_b64 instead of 2-way-conflicted
      // ds_read2st64_b64; lab A/B mixed gate_up / down -3.1 / -1.5 %, ds2_mixed -2.1 / -1.9 %,
      // w4a4 on v2x -7.5 / -5.1 %: profiles/r05/nopair/)
      // + the early-wave DMA issue on int4 tiles too (V2_I4EDMA: with the unpaired reads it now pays,
      // lab A/B w4a4 / mixed / ds2_mixed gate_up -2.7..-2.8 %, down -1.3..-3.7 %: profiles/r05/i4edma/)
      make_v2<kV2x | WO_PIPE | WO_STAG | V2_I4NOPAIR | V2_I4EDMA>("v2x_256x256_w8_b3_buf_spread_edma"),
      // round 3 (AUTO for small-batch weight-only calls): the 64-row weight-only tile at three
      // workgroups per CU (gg_wo2_kernel<.., 3>; weight-only problems only) — profiles/r03/wo2/;
      // round 4: scale groups by LDS-DMA, register constants for the code -> fp16 step, codes
      // converted where they sit, no MFMAs for row blocks past M, steady / tail loops (-10 to
      // -16 % per call at bs 512, -15 to -25 % at bs 128: profiles/r04/wo/)
      // round 6: tiles whose K stages lie in one scale group (per-channel scales) run a loop without
      // the group bookkeeping, unrolled by the ring depth (WO_PCH): ~58 fewer SALU and ~17 fewer VALU
      // per 3 stages, bit-identical; lab A/B -2.6 to -4.0 % on the per-channel bs 512 / 128 calls,
      // g128 unchanged (profiles/r06/pch/)
      make_wo2<kWo3 | WO_PCH, 3>("wo3_64x256_w8_3wg"),
#elif defined(MXMOE_LAB_FAST)
      // fast lab build (`python -m mxmoe_amd.build --lab-fast`): the product default and the
      // experiments under test only, fp16 / w8a8 bodies only
      make_v2<kV2x>("x_v2x"),
      make_v4("x_v4d_256x256_w4_1wave"),
      make_v4<1>("abl_v4d_stamp"),
      make_v3<128, 2, 3, 2>("v3_256x128_w4_dma_ring3_2wg"),  // the w4a4 AUTO kernel (A/B reference)
      make_v2<kV2x | V2_I4NOPAIR>("x_v2x_i4nopair"),
      make_v2<kV2x | V2_PLAINST>("x_v2x_plainst"),
      make_v2<kV2x | V2_TRACE>("abl_v2x_trace"),
      make_v2<kV2x | V2_TRACE | V2_TRACE_PRO>("abl_v2x_trace_pro"),
      make_v2<kV2x | V2_TRACE | V2_TRACE_DESC>("abl_v2x_trace_desc"),
      make_v2q("x_v2q"),
      make_v2q<0, 0>("x_v2q_plain"),
      make_v2q<0, 0, 1>("x_v2q_plain_fillall"),
      make_v2q<0, 16, 1>("x_v2q_fillall"),
      make_v2q<1, 0, 1>("abl_v2q_plain_fillall_trace"),
      // the small-batch weight-only tile: where its time goes (ablations: WRONG RESULTS by design)
      make_wo2<0, 3>("x_wo3_r3"),  // the round-3 loop
      make_wo2<kWo3, 3>("x_wo3"),
      make_wo2<kWo3 | WO_PCH, 3>("x_wo3_pch"),  // round 6: one-group loop (per-channel scales)
      make_wo2<kWo3, 2>("x_wo2"),
      make_wo2<kWo3 | WO_BUF, 3>("x_wo3_buf"),
      make_wo2<kWo3 | WO_ADEAD, 3>("x_wo3_adead"),
      make_wo2<kWo3 | V2_TRACE, 3>("abl_wo3_trace"),
      make_wo2<kWo3 | WO_PCH | V2_TRACE, 3>("abl_wo3_pch_trace"),  // the product loop, tile timeline
      make_wo2<kWo3 | ABL_WO_NODMA, 3>("abl_wo3_nodma"),
      make_wo2<kWo3 | ABL_WO_NOCOMPUTE, 3>("abl_wo3_nocompute"),
#else
      make_v0<T128x128, T128x128, T128x128>("v0_128x128_w4"),
      make_v0<T256x128, T256x128, T256x128>("v0_256x128_w4"),
      make_v0<T128x256, T128x256, T128x256>("v0_128x256_w4"),
      make_v2("v2_256x256_w8_dma"),
      make_v3<256, 4, 4, 3>("v3_256x256_w8_dma_ring4"),
      make_v2<kV2x>("x_v2x"),
      make_v2<kV2x | V2_I4NOPAIR>("x_v2x_i4nopair"),
      make_v2<kV2x | V2_I4NOPAIR | V2_I4EDMA>("x_v2x_i4edma"),
      // the product's default and small-batch kernels, for planner A/B runs (MXMOE_GG_XCD_PACK, _MIX)
      make_v2<kV2x | WO_PIPE | WO_STAG | V2_I4NOPAIR | V2_I4EDMA>("x_v2x_product"),
      make_wo2<kWo3, 3>("x_wo3"),
      make_wo2<kWo3 | WO_PCH, 3>("x_wo3_pch"),  // round 6: one-group loop (per-channel scales)
      // round 6: v4d, one wave per SIMD (gg_v4.h; fp16 / w8a8)
      make_v4("x_v4d_256x256_w4_1wave"),
      make_v2<kV2x | V2_PLAINST>("x_v2x_plainst"),
      make_v2<kV2x | V2_EPIPE>("x_v2x_epipe"),
      make_v2<kV2x | V2_LATEIL>("x_v2x_lateil"),
      make_v2<V2_STAGGER>("v2s_256x256_w8_dma_stagger"),
      make_v2<V2_STAGGER | V2_B3>("v2s3_256x256_w8_dma_stagger_bring3"),
      // mainloop experiments (correct results)
      make_v2<V2_STAGGER | (4 << V2_SPREAD_SHIFT)>("x_v2s_spread4"),
      make_v2<V2_STAGGER | V2_BUF | (4 << V2_SPREAD_SHIFT)>("x_v2s_buf_spread4"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | (4 << V2_SPREAD_SHIFT)>("x_v2s3_buf_spread4"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (2 << V2_SPREAD_SHIFT)>("x_v2s3_buf_edma2"),
      make_v2<V2_STAGGER | V2_BUF | V2_EARLYDMA | (2 << V2_SPREAD_SHIFT)>("x_v2s_buf_edma2"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (4 << V2_SPREAD_SHIFT)>("x_v2s3_buf_edma4"),
      make_v2p("x_v2p_256x256_w8_persistent"),
      make_v2p<1>("abl_v2p_trace"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_TRACE | (4 << V2_SPREAD_SHIFT)>("abl_v2x_trace"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | V2_TRACE | (2 << V2_SPREAD_SHIFT)>("abl_v2x_edma_trace"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | V2_STAMP | (2 << V2_SPREAD_SHIFT)>("abl_v2s3_buf_edma2_stamp"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_STAMP | (4 << V2_SPREAD_SHIFT)>("abl_v2s3_buf_sp4_stamp"),
      make_v3<128, 2, 3, 2>("v3_256x128_w4_dma_ring3_2wg"),
      // round 5: v3 at one wave per SIMD on 256 x 256 tiles (128 x 128 wave tiles, accumulators in
      // AGPRs: half the int4 widening per MFMA) — 23-33 % slower, profiles/r05/v3w/
      make_v3<256, 2, 4, 3, 4>("x_v3_256x256_w4_1wg"),
      // round 5: w4a4 on fp6 images and the fp6 MFMA (gg_f6.h; exact, 9-18 % slower than v3's int4
      // tiles on the layer calls: profiles/r05/f6/); OPT 1 unpaired reads, 2 spread DMA
      make_f6<3, 2>("f6_256x256_w8_ring3"),
      make_f6<3, 2, 1>("xf6_nopair"),
      make_f6<3, 2, 2>("xf6_spread"),
      make_f6<3, 2, 3>("xf6_nopair_spread"),
      // timing ablations of the staggered v2 (WRONG RESULTS by design; int8 tiles only)
      make_v2<V2_STAGGER | ABL_NO_DMA>("abl_v2s_nodma"),
      make_v2<V2_STAGGER | ABL_NO_EPI>("abl_v2s_noepi"),
      make_v2<V2_STAGGER | ABL_NO_DMA | ABL_NO_EPI>("abl_v2s_nodma_noepi"),
      make_v2<V2_STAGGER | V2_TRACE>("abl_v2s_trace"),
      make_v2<V2_STAGGER | ABL_DMA_HOT>("abl_v2s_dmahot"),
      // where the DMA cost goes (plain v2; int8 tiles only)
      make_v2<ABL_B_NODMA>("abl_v2_b_nodma"),
      make_v2<ABL_B_REGLOAD>("abl_v2_b_regload"),
      make_v2<ABL_B_TILED>("abl_v2_b_tiled"),
      // weight-only timing ablations (w4a16 tiles only)
      make_v2<V2_STAGGER | ABL_WO_BTILED>("abl_v2s_wo_btiled"),
      make_v2<V2_STAGGER | ABL_WO_NODMA>("abl_v2s_wo_nodma"),
      make_v2<V2_STAGGER | ABL_WO_NOCOMPUTE>("abl_v2s_wo_nocompute"),
      // weight-only experiment (correct results): v2x + the pipelined 128 / 64-row weight-only loop
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (4 << V2_SPREAD_SHIFT) | WO_PIPE>("x_v2x_wopipe"),
      make_v2<V2_STAGGER | V2_B3 | V2_BUF | V2_EARLYDMA | (4 << V2_SPREAD_SHIFT) | WO_PIPE | WO_STAG>("x_v2x_wopipe_stag"),
#endif
  };
  return v;
}

// AUTO policy: v2x (the staggered 256x256 v2 on v2s3's LDS image with the buffer-form, spread
// LDS-DMA) for every call with fp16 / bf16 / w8a8 / E4M3 / weight-only problems: same-run A/B on the
// qwen2_moe layer-11 calls, +5-11 % over v2s and +3-9 % over v2s3 at every K (the round-1/2 short-K
// rule between those two is gone: profiles/r03/lab/). int4-only sets run 256x128 tiles, 2 WG/CU
// (v3), unless they are low-fill enough to need split-K (v2 kernels only).
constexpr const char* kDefaultVariantName = "v2x_256x256_w8_b3_buf_spread_edma";
constexpr const char* kInt4Variant = "v3_256x128_w4_dma_ring3_2wg";
constexpr const char* kWoSmallVariant = "wo3_64x256_w8_3wg";
#ifdef MXMOE_LAB
constexpr const char* kF6Variant = "f6_256x256_w8_ring3";
#endif
// weight-only calls whose rows per weight byte are this small or smaller run kWoSmallVariant:
// the weight-bytes-weighted mean M over the call's problems (qwen2_moe layer 11: ~60 at bs = 128,
// ~250 at bs = 2048, ~1030 at bs = 8192, where v2x's 256-row tiles are as fast or faster)
constexpr double kWoSmallMeanRows = 512.0;
// calls of fp16 / w8a8 / w4a4 problems only (no weight-only one) take wo3 below a mean M of
// kSmallMeanRows (kSmallMeanRowsI4 with int4 problems), twice that when the call is K-skewed (its
// longest K >= 2x the weighted mean K: the qwen2_moe down call, whose shared expert has 4x the
// routed K — few long tiles the general kernels balance poorly). Measured on qwen2_moe layer 11
// (mean M ~ bs / 8; profiles/r03/wo2/wo3_fp16_w8a8.jsonl, wo3_w4a4_mixed.jsonl, wo3_mid.jsonl):
// gate_up wins to bs 512 (fp16 -3.5 .. w4a4 +33 %) and 768 with int4, down calls to bs 1024 (fp16)
// / 1536 (int4), the general kernels beyond.
constexpr double kSmallMeanRows = 80.0;
constexpr double kSmallMeanRowsI4 = 112.0;
constexpr double kSplitCUs = 256.0;  // MI355X compute units: the planner's notion of "one CU's share"

int variant_index(const char* name) {
  for (size_t i = 0; i < variants().size(); ++i)
    if (!strcmp(variants()[i].name, name)) return (int)i;
  return 0;
}

int qtype_of(int a_bits, int w_bits, int gsize, int sym, int fmt, int* qt) {
  fmt &= 0xFF;  // (epilogue flags, MXMOE_GG_EPI_*, live above the operand format)
  if (fmt == MXMOE_GG_FMT_E4M3) {  // w8a8_g-1_sym_E4M3 (tile_config.py:45, 104-106, 192)
    if (a_bits == 8 && w_bits == 8 && gsize == -1 && sym) {
      *qt = QT_F8;
      return MXMOE_GG_OK;
    }
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported: w%da%d_g%d_%s_E4M3 (only w8a8_g-1_sym_E4M3)",
                w_bits, a_bits, gsize, sym ? "sym" : "asym");
  }
  if (fmt == MXMOE_GG_FMT_BF16) {  // bf16 (tile_config.py:42, 99-102)
    if (a_bits == 16 && w_bits == 16) {
      *qt = QT_BF16;
      return MXMOE_GG_OK;
    }
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported: w%da%d bf16 (only 16-bit bf16 operands)", w_bits,
                a_bits);
  }
#ifdef MXMOE_LAB
  if (fmt == MXMOE_GG_FMT_F6) {  // w4a4_g-1_sym with fp6 images of the int4 codes (mxmoe_gg_pack_f6)
    if (a_bits == 4 && w_bits == 4 && gsize == -1 && sym) {
      *qt = QT_I4F6;
      return MXMOE_GG_OK;
    }
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported: w%da%d_g%d_%s as fp6 images (only w4a4_g-1_sym)",
                w_bits, a_bits, gsize, sym ? "sym" : "asym");
  }
#endif
  if (fmt != MXMOE_GG_FMT_DEFAULT) return fail(MXMOE_GG_ERR_UNSUPPORTED, "unknown operand format %d", fmt);
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
  if (a_bits == 4 && w_bits == 4 && gsize == 128 && sym) {  // w4a4_g128_sym (cta_gemm.cuh:610-772)
    *qt = QT_I4G;
    return MXMOE_GG_OK;
  }
  if (a_bits == 16 && (w_bits == 2 || w_bits == 4 || w_bits == 8)) {  // weight-only; group size checked per problem
    *qt = w_bits == 2 ? QT_W2A16 : w_bits == 4 ? QT_W4A16 : QT_W8A16;
    return MXMOE_GG_OK;
  }
  return fail(MXMOE_GG_ERR_UNSUPPORTED, "quant type not supported: w%da%d_g%d_%s", w_bits, a_bits, gsize,
              sym ? "sym" : "asym");
}

bool is_weightonly(int qt) { return qt == QT_W4A16 || qt == QT_W8A16 || qt == QT_W2A16; }
bool is_float16(int qt) { return qt == QT_F16 || qt == QT_BF16; }  // 16-bit operands, no scales

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct HostProblem {
  const void *A, *B, *SA, *SB;
  void* C;
  int M, N, K, a_bits, w_bits, gsize, sym;
  int64_t lda, ldb, ldc;  // 16-bit words, 0 = dense
  int fmt;                // MXMOE_GG_FMT_*
};

// Workspace: [GGMeta x P][ptr_A x P][ptr_B x P][ptr_SA x P][ptr_SB x P][ptr_C x P][TileDesc x grid]
// workspace: plan table | 5 pointer columns | tile table | split-K counters (one per tile slot,
// zero between launches) | split-K slabs
struct WsLayout {
  size_t meta, ptr, tiles, counters, slabs, total;
};
WsLayout ws_layout(int P, int grid, int slabs) {
  WsLayout l;
  l.meta = align_up((size_t)std::max(P, 1) * sizeof(GGMeta), 256);
  l.ptr = align_up((size_t)std::max(P, 1) * sizeof(void*), 256);
  l.tiles = align_up((size_t)std::max(grid, 1) * sizeof(TileDesc), 256);
  l.counters = slabs ? align_up((size_t)grid * sizeof(int32_t), 256) : 0;
  l.slabs = (size_t)slabs * SPLITK_SLAB_BYTES;
  l.total = l.meta + 5 * l.ptr + l.tiles + l.counters + l.slabs;
  return l;
}

// Validate one problem and fill its table row.
// Weight-only WxA16: A fp16 [M][K], B codes [N][K * w_bits / 8] (mxmoe_gg_repack_weightonly
// layout), scale_b = scale / zp in the reference permute_scale layout; K in 64-element stages.
int build_meta_weightonly(const HostProblem& p, int idx, int qt, const Variant& v, bool check_ptrs, GGMeta* m) {
  if (p.K % 64) return fail(MXMOE_GG_ERR_INVALID, "problem %d: weight-only needs K %% 64 == 0 (K=%d)", idx, p.K);
  if (p.gsize != -1 && (p.gsize <= 0 || p.gsize % 64 || p.K % p.gsize))
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "problem %d: weight-only group size %d must be -1 or a multiple of 64 dividing K=%d",
                idx, p.gsize, p.K);
  if (p.N % 8 != 0) return fail(MXMOE_GG_ERR_INVALID, "problem %d: N=%d must be a multiple of 8", idx, p.N);
  const bool silu = (p.fmt & MXMOE_GG_EPI_SILU_MUL) != 0;  // (build_meta checked N % 32 and the variant)
  const int64_t arow = (int64_t)p.K * 2, brow = (int64_t)p.K * p.w_bits / 8;
  const int64_t lda_b = p.lda ? p.lda * 2 : arow;
  const int64_t ldb_b = p.ldb ? p.ldb * 2 : brow;
  const int64_t ncols = silu ? p.N / 2 : p.N;  // columns of C
  const int64_t ldc = p.ldc ? p.ldc : ncols;
  if (lda_b < arow || ldb_b < brow || (lda_b % 16) || (ldb_b % 16))
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: lda/ldb must be >= K row and a multiple of 8 words", idx);
  if (ldc < ncols || (ldc % 8))
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: ldc must be >= %s and a multiple of 8", idx, silu ? "N / 2" : "N");
  if (check_ptrs && p.M > 0 && p.N > 0) {
    if (!p.A || !p.B || !p.C) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL A/B/C", idx);
    if (!p.SB) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL scale pointer (weight-only scale_b)", idx);
    if (((uintptr_t)p.A | (uintptr_t)p.B | (uintptr_t)p.C) & 15)
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: A/B/C must be 16-byte aligned", idx);
    if (((uintptr_t)p.SB) & (p.sym ? 1 : 3))
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: scales must be %d-byte aligned", idx, p.sym ? 2 : 4);
  }
  memset(m, 0, sizeof(*m));
  m->M = p.M;
  m->N = p.N;
  m->K = p.K;
  m->qtype = qt;
  m->tiles_n = (p.N + v.geom[qt].bn - 1) / v.geom[qt].bn;
  m->kbytes = (int32_t)arow;
  m->reserved = p.gsize == -1 ? std::max(1, p.K / 64) : p.gsize / 64;  // 64-K stages per scale group
  m->reserved2 = (p.sym ? 1 : 0) | (silu ? META_SILU : 0);
  m->lda_b = lda_b;
  m->ldb_b = ldb_b;
  m->ldc = ldc;
  return MXMOE_GG_OK;
}

int build_meta(const HostProblem& p, int idx, const Variant& v, bool check_ptrs, GGMeta* m) {
  if (p.M < 0 || p.N < 0 || p.K < 0) return fail(MXMOE_GG_ERR_INVALID, "problem %d: negative shape", idx);
  int qt = 0;
  int st = qtype_of(p.a_bits, p.w_bits, p.gsize, p.sym, p.fmt, &qt);
  if (st) return fail(st, "problem %d: %s", idx, g_last_error.c_str());
  if (v.geom[qt].bn == 0)
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "problem %d: variant %s does not implement w%da%d (quant type not supported)",
                idx, v.name, p.w_bits, p.a_bits);
  const bool silu = (p.fmt & MXMOE_GG_EPI_SILU_MUL) != 0;
  if (p.fmt & ~(0xFF | MXMOE_GG_EPI_SILU_MUL)) return fail(MXMOE_GG_ERR_INVALID, "problem %d: unknown fmt flags %#x", idx, p.fmt);
  if (silu && !(qt == QT_F16 || qt == QT_I8 || qt == QT_I4 || (is_weightonly(qt) && v.silu_wo)))
    return fail(MXMOE_GG_ERR_UNSUPPORTED,
                "problem %d: the SiLU epilogue needs fp16, w8a8_g-1_sym or w4a4_g-1_sym (weight-only: the small-batch "
                "kernel wo3)", idx);
  if (silu && !has_silu_epilogue(v))
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "problem %d: variant %s has no SiLU epilogue", idx, v.name);
  if (silu && p.N % 32) return fail(MXMOE_GG_ERR_INVALID, "problem %d: the SiLU epilogue needs N %% 32 == 0 (N=%d)", idx, p.N);
  if (is_weightonly(qt)) return build_meta_weightonly(p, idx, qt, v, check_ptrs, m);
  const int abits = is_float16(qt) ? 16 : p.a_bits;
  const int64_t kbits = (int64_t)p.K * abits;  // (fp6 images: K of the int4 codes they encode)
  if (kbits % 128 != 0)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: K=%d must be a multiple of %d for %d-bit data (16-B rows)", idx,
                p.K, (int)(128 / abits), abits);
  if (v.k_stage_bytes && (kbits / 8) % v.k_stage_bytes != 0)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: variant %s needs K*bits/8 to be a multiple of %d bytes (K=%d)",
                idx, v.name, v.k_stage_bytes, p.K);
  if (qt == QT_I4G && p.K % 128 != 0)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: w4a4_g128 needs K %% 128 == 0 (K=%d)", idx, p.K);
  if (qt != QT_F16 && qt != QT_BF16 && qt != QT_F8 && p.K > 131072)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: K=%d exceeds the exact int32 accumulation bound 131072", idx, p.K);
  if (p.N % 8 != 0) return fail(MXMOE_GG_ERR_INVALID, "problem %d: N=%d must be a multiple of 8", idx, p.N);
  // fp6 images: 96 B per K-128 block, K padded to whole blocks (mxmoe_gg_pack_f6)
#ifdef MXMOE_LAB
  const int64_t kbytes = qt == QT_I4F6 ? (int64_t)MXMOE_GG_F6_ROW_BYTES(p.K) : kbits / 8;
#else
  const int64_t kbytes = kbits / 8;
#endif
  const int64_t lda_b = p.lda ? p.lda * 2 : kbytes;
  const int64_t ldb_b = p.ldb ? p.ldb * 2 : kbytes;
  const int64_t ncols = silu ? p.N / 2 : p.N;  // columns of C
  const int64_t ldc = p.ldc ? p.ldc : ncols;
  if (lda_b < kbytes || ldb_b < kbytes || (lda_b % 16) || (ldb_b % 16))
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: lda/ldb must be >= K row and a multiple of 8 words", idx);
  // the buffer-form LDS-DMA addresses a 256-row tile with 32-bit offsets below 2^31
  if (lda_b >= (int64_t)1 << 23 || ldb_b >= (int64_t)1 << 23)
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: A / B row strides must be below 8 MiB", idx);
  if (ldc < ncols || (ldc % 8))
    return fail(MXMOE_GG_ERR_INVALID, "problem %d: ldc must be >= %s and a multiple of 8", idx, silu ? "N / 2" : "N");
  if (check_ptrs && p.M > 0 && p.N > 0) {  // empty problems are dropped by the planner
    if (!p.A || !p.B || !p.C) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL A/B/C", idx);
    if (!is_float16(qt) && (!p.SA || !p.SB)) return fail(MXMOE_GG_ERR_INVALID, "problem %d: NULL scale pointer", idx);
    if (((uintptr_t)p.A | (uintptr_t)p.B | (uintptr_t)p.C) & 15)
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: A/B/C must be 16-byte aligned", idx);
    if (!is_float16(qt) && (((uintptr_t)p.SA | (uintptr_t)p.SB) & 1))
      return fail(MXMOE_GG_ERR_INVALID, "problem %d: scales must be 2-byte aligned", idx);
  }
  memset(m, 0, sizeof(*m));
  m->M = p.M;
  m->N = p.N;
  m->K = p.K;
  m->qtype = qt;
  m->tiles_n = (p.N + v.geom[qt].bn - 1) / v.geom[qt].bn;
  m->kbytes = (int32_t)kbytes;
  m->reserved = qt == QT_I4G ? p.K / 128 : 0;  // w4a4 g128: scale groups
  m->reserved2 = silu ? META_SILU : 0;
  m->lda_b = lda_b;
  m->ldb_b = ldb_b;
  m->ldc = ldc;
  return MXMOE_GG_OK;
}

struct Plan {
  std::vector<GGMeta> meta;     // table rows (planned problems only)
  std::vector<int> order;       // table row -> caller's problem index
  std::vector<TileDesc> tiles;  // indexed by blockIdx
  int total_tiles = 0;
  int launch_grid = 0;          // workgroups launched (= tiles.size() unless persistent)
  int slabs = 0;                // split-K partial slabs
  int tail_slabs = 0;           // of which for the tail split (plan_host)
};

// Tile generation + scheduling.
//  1. per problem: m-tiles of the variant's height (v2: 256-row tiles while > tail_bm rows remain,
//     then one tail_bm (128) or tail2_bm (64) tile), n-tiles of width bn; 4-m-tile bands, n-major
//     inside a band, so 32 consecutive tiles form a ~4 x 8 block sharing A rows and B columns;
//  2. problems by descending per-tile cost (K bytes x tile area x MFMA passes), longest first;
//  3. XCD regions: a problem of >= 8 chunks of tiles (the shared expert at large batch) is cut
//     into 8 rectangles of its tile grid, one per XCD, at the head of that XCD's queue (region_of);
//  4. the rest is cut into chunks of about `chunk` tiles that do not straddle problems; each chunk
//     in turn joins the queue of the XCD with the least modelled time so far (tile_time); XCD x's
//     i-th tile is blockIdx 8 i + x (blocks b and b + 8 share an XCD under the round-robin
//     dispatch; placement affects speed and HBM traffic only, never results).
int plan_host(const std::vector<HostProblem>& probs, int variant, bool check_ptrs, Plan* plan) {
  const Variant& v = variants()[variant];
  const int P = (int)probs.size();
  std::vector<GGMeta> all(P);
  for (int i = 0; i < P; ++i) {
    int st = build_meta(probs[i], i, v, check_ptrs, &all[i]);
    if (st) return st;
  }
  std::vector<int> order;
  for (int i = 0; i < P; ++i)
    if (probs[i].M > 0 && probs[i].N > 0) order.push_back(i);
  // K stages of a problem in its tile body (v2: 128 B per stage; weight-only: 64 elements)
  auto stages_of = [&](const GGMeta& m) {
    if (is_weightonly(m.qtype)) return m.K / 64;
    return (m.kbytes + v.geom[m.qtype].bkb - 1) / v.geom[m.qtype].bkb;
  };
  auto full_tile_cost = [&](int i) {
    const GGMeta& m = all[i];
    // int4: 2 MFMA passes per staged byte; g128 adds the per-group f32 fold (~25 %); fp6 images:
    // one fp6 MFMA (the int8 one's cycles) per 96 B of K-128
    const double passes = m.qtype == QT_I4 ? 2.0 : m.qtype == QT_I4G ? 2.5 : m.qtype == QT_I4F6 ? 128.0 / 96 / 2 : 1.0;
    return passes * (double)m.kbytes * v.geom[m.qtype].bm * v.geom[m.qtype].bn;
  };
  // m-tiles of a problem: (m0, class); v2 classes 256 / 128 / 64 rows (see Variant::tail_bm)
  auto class_rows = [&](int cls, const TileGeom& g) { return cls == 0 ? g.bm : cls == 1 ? v.tail_bm : v.tail2_bm; };
  auto m_tiles = [&](const GGMeta& m) {
    const TileGeom& g = v.geom[m.qtype];
    std::vector<std::pair<int, int>> mt;
    for (int m0 = 0; m0 < m.M;) {
      const int rem = m.M - m0;
      const bool small_class = is_float16(m.qtype) || is_weightonly(m.qtype);
      if (v.kind != Kind::V0 && v.tail2_bm && small_class && rem <= v.tail2_bm) {
        mt.push_back({m0, 2});
        m0 += v.tail2_bm;
      } else if (v.kind != Kind::V0 && v.tail_bm && rem <= v.tail_bm) {
        mt.push_back({m0, 1});
        m0 += v.tail_bm;
      } else {
        mt.push_back({m0, 0});
        m0 += g.bm;
      }
    }
    return mt;
  };
  // split-K (v2 kernels): a problem whose largest tile is far longer than one CU's share of the
  // whole call (low-fill calls: small batches, long-K shared experts, per-rank work lists) has its
  // tiles cut into split[i] K slices of >= 4 stages each, at most 8
  std::vector<int> split(P, 1);
  if (v.kind == Kind::V2) {
    double total = 0;
    std::vector<double> biggest(P, 0.0);
    for (int i : order) {
      const GGMeta& m = all[i];
      const TileGeom& g = v.geom[m.qtype];
      const double per_row = full_tile_cost(i) / g.bm;
      for (const auto& t : m_tiles(m)) {
        const double c = per_row * class_rows(t.second, g);
        total += c * m.tiles_n;
        biggest[i] = std::max(biggest[i], c);
      }
    }
    const double share = total / (kSplitCUs * v.chunk / 32);  // workgroup slots: CUs x workgroups per CU
    const char* rmul_env = planner_knob("MXMOE_GG_SPLIT_RATIO_MUL");  // lab A/B: scale the ratio
    const double rmul = rmul_env ? atof(rmul_env) : 1.0;
    for (int i : order) {
      const double ratio = rmul * biggest[i] / std::max(share, 1.0);
      // (w4a4 g128 never splits: summing f32 partial folds would change the rounding)
      if (ratio > 2.0 && all[i].qtype != QT_I4G) split[i] = std::max(1, std::min({8, (int)ratio, stages_of(all[i]) / 4}));
    }
    // lab A/B switch: every problem split into at least S K slices (where it has >= 4 S stages)
    const char* sall = planner_knob("MXMOE_GG_SPLITK_ALL");
    if (sall && atoi(sall) > 1)
      for (int i : order)
        if (all[i].qtype != QT_I4G)
          split[i] = std::max(split[i], std::max(1, std::min({8, atoi(sall), stages_of(all[i]) / 4})));
  }
  // Tile time model (per K stage, in "bytes": one stage's LDS-DMA bytes or its MFMA work at the
  // fp16 rate of 128 flop/B, whichever is larger, plus a fixed 24 KiB-equivalent per stage).
  // Fitted to the tile timelines (profiles/r01/session3/trace_bs512.jsonl): 64-row /
  // 256-row tile time ratios 1.3 (fp16) and 2.1 (w4a16), where tile area alone says 4.
  auto stage_time = [&](const GGMeta& m, int cls) {
    const TileGeom& g = v.geom[m.qtype];
    const double rows = class_rows(cls, g), cols = g.bn;
    double bytes, equiv;
    if (is_weightonly(m.qtype)) {  // 64 K elements per stage, fp16 A
      bytes = rows * 128 + cols * 64 * (m.qtype == QT_W2A16 ? 2 : m.qtype == QT_W4A16 ? 4 : 8) / 8.0;
      equiv = 2.0 * rows * cols * 64 / 128;
    } else {
      const double kel = m.qtype == QT_I4F6 ? 128.0
                       : g.bkb * 8.0 / (is_float16(m.qtype) ? 16 : (m.qtype == QT_I8 || m.qtype == QT_F8) ? 8 : 4);
      const double rate = is_float16(m.qtype) ? 128 : m.qtype == QT_I4F6 ? 512 : 256, fold = m.qtype == QT_I4G ? 1.25 : 1.0;
      bytes = (rows + cols) * g.bkb;
      equiv = 2.0 * rows * cols * kel / rate * fold;
    }
    return std::max(bytes, equiv) + 24576.0;
  };
  // problems by the modelled time of their first (tallest) tile, longest first
  std::vector<double> tile_cost(P, 0.0);
  for (int i : order) tile_cost[i] = stage_time(all[i], m_tiles(all[i])[0].second) * stages_of(all[i]) / split[i];
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return tile_cost[a] > tile_cost[b]; });

  // m-tiles per band (n-major inside a band): a 32-tile chunk is band x (32 / band) tiles
  const char* band_env = planner_knob("MXMOE_GG_BAND");  // A/B switch (default 4)
  const size_t band = band_env && atoi(band_env) > 0 ? (size_t)atoi(band_env) : 4;
  const char* ngroup_env = planner_knob("MXMOE_GG_NGROUP");  // A/B switch (default 1)
  const int ngroup = ngroup_env && atoi(ngroup_env) > 0 ? atoi(ngroup_env) : 1;
  plan->meta.clear();
  plan->order = order;
  plan->slabs = 0;
  plan->tail_slabs = 0;
  const int chunk = v.chunk;
  // XCD regions. Within one XCD, consecutive tiles run together (the XCD hands each freed CU its
  // next block), so a band's A rows and B columns are re-read from that XCD's L2 while they are
  // hot; but under chunked LPT a 4-m-tile band of the 44 n-tile shared expert lands on ~5 XCDs and
  // each fetches the band's A panels again (and every band its B panels): 528 MB of panel reads
  // for 78 MB of operands at bs=8192. One rectangle per XCD (r m-tiles x c n-tiles, enumerated in
  // bands of `band` along the cheaper axis) reads r A panels + ceil(r / band) * c B panels (or the
  // transpose) — the split of the grid into 8 rectangles is chosen to minimise that sum.
  // placement: after the chunked tiles (default; measured 1-5 % faster than at the queue head on the
  // w8a8 gate_up / down / mixed calls, profiles/r02/region/)
  const char* region_env = planner_knob("MXMOE_GG_REGION");  // A/B switch: 0 off, 1 queue head, 2 tail (default)
  const bool regions_on = !(region_env && region_env[0] == '0');
  const bool regions_last = !(region_env && region_env[0] == '1');
  const char* rot_env = planner_knob("MXMOE_GG_REGION_ROT");  // A/B switch (default off)
  const bool region_rot = rot_env && rot_env[0] == '1';
  const char* align_env = planner_knob("MXMOE_GG_ALIGN");  // A/B switch: problem-aligned chunks (default on)
  const bool align_on = !(align_env && align_env[0] == '0');
  struct Region {
    int gm = 0, gn = 0, r = 0, c = 0;
    bool nband = false;  // true: bands of n-tiles, m-major inside
  };
  auto region_of = [&](int i, Region* out) {
    const GGMeta& m = all[i];
    const int mt = (int)m_tiles(m).size(), nt = m.tiles_n;
    if (!regions_on || v.kind != Kind::V2 || split[i] != 1 || (int64_t)mt * nt < 8 * (int64_t)chunk) return false;
    const TileGeom& g = v.geom[m.qtype];
    const double a_panel = (double)g.bm * m.kbytes, b_panel = (double)g.bn * m.K * probs[i].w_bits / 8.0;
    double best = 0;
    for (int gm = 1; gm <= 8; gm *= 2) {
      const int gn = 8 / gm;
      if (mt < gm || nt < gn) continue;
      const int r = (mt + gm - 1) / gm, c = (nt + gn - 1) / gn;
      // every region non-empty and within 25 % of the largest (the LPT fill evens out the rest)
      const int r_last = mt - (gm - 1) * r, c_last = nt - (gn - 1) * c;
      if (r_last <= 0 || c_last <= 0 || 4 * (int64_t)r_last * c_last < 3 * (int64_t)r * c) continue;
      const int b = (int)band;
      const double mband = r * a_panel + (double)((r + b - 1) / b) * c * b_panel;
      const double nband = c * b_panel + (double)((c + b - 1) / b) * r * a_panel;
      const double cost = std::min(mband, nband);
      if (out->gm == 0 || cost < best) {
        *out = Region{gm, gn, r, c, nband < mband};
        best = cost;
      }
    }
    return out->gm != 0;
  };
  int groups = 0, n_region = 0;
  bool region_a16 = false;
  std::vector<TileDesc> seq;                // chunked tiles
  std::vector<int> seq_end;                 // per seq tile: end of its problem's run in seq
  std::vector<std::vector<TileDesc>> region_tiles(8);  // per XCD
  for (int row = 0; row < (int)order.size(); ++row) {
    GGMeta m = all[order[row]];
    const TileGeom& g = v.geom[m.qtype];
    const std::vector<std::pair<int, int>> mt = m_tiles(m);  // (m0, cls)
    m.tile_begin = (int32_t)seq.size();
    const int nt = m.tiles_n, S = split[order[row]], nst = stages_of(m);
    Region rg;
    if (region_of(order[row], &rg)) {
      ++n_region;
      region_a16 = region_a16 || probs[order[row]].a_bits == 16;
      for (int x = 0; x < 8; ++x) {
        const int mb0 = (x / rg.gn) * rg.r, mb1 = std::min((int)mt.size(), mb0 + rg.r);
        const int nb0 = (x % rg.gn) * rg.c, nb1 = std::min(nt, nb0 + rg.c);
        auto put = [&](int mi, int n) {
          region_tiles[x].push_back(TileDesc{row, mt[mi].first, n * g.bn, mt[mi].second, 0, nst, -1, -1});
        };
        // (MXMOE_GG_REGION_ROT: XCD x starts its sweep x/8 of the way along the swept axis, so the
        // XCDs do not all stream the same panels at the same time)
        const int span_n = nb1 - nb0, span_m = mb1 - mb0;
        const int rot_n = region_rot && span_n > 0 ? (x * span_n / 8) : 0;
        const int rot_m = region_rot && span_m > 0 ? (x * span_m / 8) : 0;
        if (rg.nband) {
          for (int nb = nb0; nb < nb1; nb += (int)band)
            for (int k = 0; k < span_m; ++k) {
              const int mi = mb0 + (k + rot_m) % span_m;
              for (int n = nb; n < std::min(nb1, nb + (int)band); ++n) put(mi, n);
            }
        } else {
          for (int mb = mb0; mb < mb1; mb += (int)band)
            for (int k = 0; k < span_n; ++k) {
              const int n = nb0 + (k + rot_n) % span_n;
              for (int mi = mb; mi < std::min(mb1, mb + (int)band); ++mi) put(mi, n);
            }
        }
      }
      plan->meta.push_back(m);
      continue;
    }
    // (lab A/B, MXMOE_GG_NGROUP = G: inside a band, n-tiles in groups of G, m-major inside a group —
    // G = 1 is the default n-major order, G >= tiles_n m-major)
    for (size_t mb = 0; mb < mt.size(); mb += band)
      for (int ng = 0; ng < nt; ng += ngroup)
        for (size_t mi = mb; mi < std::min(mt.size(), mb + band); ++mi)
          for (int n = ng; n < std::min(nt, ng + ngroup); ++n) {
          if (S == 1) {
            seq.push_back(TileDesc{row, mt[mi].first, n * g.bn, mt[mi].second, 0, nst, -1, -1});
            continue;
          }
          const int grp = groups++, slab = plan->slabs;
          plan->slabs += S;
          for (int k = 0; k < S; ++k)  // slices of one tile are consecutive: they start together
            seq.push_back(TileDesc{row, mt[mi].first, n * g.bn, mt[mi].second | (k << 8) | (S << 16),
                                   k * nst / S, (k + 1) * nst / S, slab, grp});
        }
    seq_end.resize(seq.size(), (int)seq.size());
    plan->meta.push_back(m);
  }
  size_t T_head = 0;
  for (const auto& h : region_tiles) T_head += h.size();
  const int T = (int)(seq.size() + T_head);
  if (T > (1 << 28)) return fail(MXMOE_GG_ERR_INVALID, "too many tiles (%d)", T);
  auto tile_time = [&](const TileDesc& td) {
    return stage_time(plan->meta[td.prob], td.cls & 0xFF) * (td.ks1 - td.ks0);
  };
  // XCD queues (XCD x's i-th tile is block 8 i + x). Chunks in LPT order: full chunks join the
  // XCD queue with the least modelled time; the last 16 chunks' worth of tiles go in chunks of
  // `tail_chunk`, each to the XCD whose simulated finish grows least (ties: least total time) —
  // every XCD simulated as `chunk` workgroup slots taking its queue in order, as the hardware
  // hands a freed slot the XCD's next block. Plain round-robin chunks let a low-fill call's few
  // long tiles pile onto 2-3 XCDs (bs=512: per-XCD busy time 40 % apart).
  struct XcdSim {
    std::vector<double> slot;  // min-heap of slot free times
    double finish = 0, load = 0;
    void add(double t) {
      std::pop_heap(slot.begin(), slot.end(), std::greater<double>());
      slot.back() += t;
      finish = std::max(finish, slot.back());
      std::push_heap(slot.begin(), slot.end(), std::greater<double>());
      load += t;
    }
  };
  std::vector<XcdSim> sim(8);
  for (auto& x : sim) x.slot.assign(chunk, 0.0);
  std::vector<std::vector<int>> queue(8);  // indices into `all_tiles`: region tiles first, then chunks
  std::vector<TileDesc> all_tiles(seq);
  auto put_regions = [&]() {
    for (int x = 0; x < 8; ++x)
      for (const TileDesc& td : region_tiles[x]) {
        sim[x].add(tile_time(td));
        queue[x].push_back((int)all_tiles.size());
        all_tiles.push_back(td);
      }
  };
  const int TS = (int)seq.size();
  // XCD packing (lab A/B: MXMOE_GG_XCD_PACK = 1 region tiles at the queue head,
  // 2 at the tail). A call with region problems (the shared expert) and small ones (routed experts):
  // every small problem goes WHOLE to one XCD — LPT over the problems' modelled loads, so its A / B
  // panels live in one L2 — and the region problems' tiles, taken in rectangle order, are the filler
  // that levels the XCDs: tile by tile to the XCD of least modelled load, then cut into consecutive
  // pieces (XCD x's piece overlaps its rectangle, so the panel reuse of the rectangles is kept).
  // Default (pack 4, product): packing for the MoE call shape — ONE region problem (the shared expert)
  // beside >= 8 whole small problems — with the region tiles at the queue head when they are the long
  // ones (down: K 4x the routed K; LPT) or when the region problem's A is 16-bit (its panels stream
  // twice the bytes per flop: the fp16 gate_up call's head placement cut its counter bytes 2.97 ->
  // 2.35 GB and ran 2.4 % faster, where w8a8 gate_up at the head ran 4 % slower, profiles/r06/pack/;
  // an arithmetic-intensity cut in its place also sent the int calls of small batches to the head,
  // 3-8 % slower at bs 2048, profiles/r06/plan3/); every other call keeps the chunked placement. Lab A/B:
  // MXMOE_GG_XCD_PACK = 0 off, 1 always head, 2 always tail, 3 head only for long region tiles.
  const char* pack_env = planner_knob("MXMOE_GG_XCD_PACK");
  const int pack = pack_env ? atoi(pack_env) : 4;
  bool packed = false;
  int n_small = 0;
  for (int s0 = 0; s0 < TS; s0 = seq_end[s0]) ++n_small;
  const bool moe_shape = n_region == 1 && n_small >= 8;
  if (pack > 0 && T_head > 0 && v.kind == Kind::V2 && !v.persistent && (pack != 4 || moe_shape)) {
    std::vector<std::pair<int, int>> runs;  // [s0, s1) of one problem's tiles in seq
    for (int s0 = 0; s0 < TS; s0 = seq_end[s0]) runs.push_back({s0, seq_end[s0]});
    std::vector<double> rl(runs.size(), 0.0);
    for (size_t r = 0; r < runs.size(); ++r)
      for (int s = runs[r].first; s < runs[r].second; ++s) rl[r] += tile_time(seq[s]);
    std::vector<int> ro(runs.size());
    for (size_t r = 0; r < ro.size(); ++r) ro[r] = (int)r;
    std::stable_sort(ro.begin(), ro.end(), [&](int a, int b) { return rl[a] > rl[b]; });
    double load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    std::vector<std::vector<int>> small_q(8);
    for (int r : ro) {
      int x = 0;
      for (int y = 1; y < 8; ++y)
        if (load[y] < load[x]) x = y;
      load[x] += rl[r];
      for (int s = runs[r].first; s < runs[r].second; ++s) small_q[x].push_back(s);
    }
    std::vector<TileDesc> big;
    for (int x = 0; x < 8; ++x) big.insert(big.end(), region_tiles[x].begin(), region_tiles[x].end());
    int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (const TileDesc& td : big) {
      int x = 0;
      for (int y = 1; y < 8; ++y)
        if (load[y] < load[x]) x = y;
      load[x] += tile_time(td);
      ++cnt[x];
    }
    // the XCD's queue as its slots take it: region tiles first (pack 1) or last, and the queue's last
    // 2 * chunk tiles longest first (the tail tiles of the routed bands are the short ones: LPT at the
    // end evens the slots' finish; earlier tiles keep the band order)
    // pack 3: at the head when the region tiles are the long ones (the down call's shared expert, 4x
    // the routed K: LPT), at the tail otherwise (gate_up: every tile the same length)
    bool head = pack == 1;
    if (pack >= 3) {
      double tb = 0, ts = 0;
      for (const TileDesc& td : big) tb += tile_time(td);
      for (int e = 0; e < TS; ++e) ts += tile_time(seq[e]);
      head = !big.empty() && TS > 0 && tb / big.size() >= 1.5 * ts / TS;
      if (pack == 4) head = head || region_a16;  // a 16-bit region problem (fp16 / bf16 / weight-only A)
    }
    // XCD x's region tiles: first its own rectangle (region_tiles[x], in band order) up to cnt[x]; the
    // rectangles' surplus tails then fill the XCDs that take more than their own (a piece stays one
    // rectangle plus at most a band's worth of a neighbour: the panel reuse the rectangles bought)
    std::vector<size_t> rb(9, 0);
    for (int x = 0; x < 8; ++x) rb[x + 1] = rb[x] + region_tiles[x].size();
    std::vector<std::vector<int>> pieces(8);
    auto assign_pieces = [&]() {
      std::vector<int> pool;
      for (int x = 0; x < 8; ++x) {
        pieces[x].clear();
        const size_t own = rb[x + 1] - rb[x], take = std::min(own, (size_t)cnt[x]);
        for (size_t k = 0; k < own; ++k) (k < take ? pieces[x] : pool).push_back((int)(rb[x] + k));
      }
      size_t p = 0;
      for (int x = 0; x < 8; ++x)
        while ((int)pieces[x].size() < cnt[x] && p < pool.size()) pieces[x].push_back(pool[p++]);
    };
    auto build_q = [&](int x, std::vector<int>* q) {
      q->clear();
      std::vector<int> bq;
      for (int k : pieces[x]) bq.push_back(-1 - k);  // (big tiles: -1 - index)
      if (head) *q = bq;
      q->insert(q->end(), small_q[x].begin(), small_q[x].end());
      if (!head) q->insert(q->end(), bq.begin(), bq.end());
      const size_t n = q->size(), tail = std::min(n, (size_t)(2 * chunk));
      auto tt = [&](int e) { return e < 0 ? tile_time(big[-1 - e]) : tile_time(seq[e]); };
      std::stable_sort(q->end() - tail, q->end(), [&](int a, int b) { return tt(a) > tt(b); });
    };
    auto finish_of = [&](const std::vector<int>& q) {
      XcdSim xs;
      xs.slot.assign(chunk, 0.0);
      for (int e : q) xs.add(e < 0 ? tile_time(big[-1 - e]) : tile_time(seq[e]));
      return xs.finish;
    };
    // local search: move one region tile from the XCD that finishes last to the one that finishes
    // first while the modelled makespan drops (the loads above are level; the slots' finish is not)
    std::vector<std::vector<int>> q(8);
    double fin[8];
    auto rebuild = [&]() {
      assign_pieces();
      for (int x = 0; x < 8; ++x) {
        build_q(x, &q[x]);
        fin[x] = finish_of(q[x]);
      }
    };
    rebuild();
    // (compared as the sorted finish vector, latest first: a move that takes one of several XCDs off
    // the makespan counts as a gain)
    auto key = [&]() {
      std::vector<double> f(fin, fin + 8);
      std::sort(f.begin(), f.end(), std::greater<double>());
      return f;
    };
    for (int it = 0; it < 128; ++it) {
      int hi = 0, lo = 0;
      for (int x = 1; x < 8; ++x) {
        if (fin[x] > fin[hi]) hi = x;
        if (fin[x] < fin[lo]) lo = x;
      }
      if (cnt[hi] == 0 || hi == lo) break;
      const std::vector<double> before = key();
      --cnt[hi];
      ++cnt[lo];
      rebuild();
      if (!(key() < before)) {  // no gain: undo and stop
        ++cnt[hi];
        --cnt[lo];
        rebuild();
        break;
      }
    }
    const int base = (int)all_tiles.size();
    all_tiles.insert(all_tiles.end(), big.begin(), big.end());
    for (int x = 0; x < 8; ++x) {
      queue[x].clear();
      for (int e : q[x]) queue[x].push_back(e < 0 ? base + (-1 - e) : e);
    }
    packed = true;
  }
  if (!regions_last && !packed) put_regions();
  const char* tc_env = planner_knob("MXMOE_GG_TAIL_CHUNK");  // A/B switch: tail chunk size (default 16)
  const int tail_chunk = tc_env && atoi(tc_env) > 0 ? atoi(tc_env) : 16;
  const char* rr_env = planner_knob("MXMOE_GG_XCD_RR");  // A/B switch: plain round-robin chunks
  const bool round_robin = rr_env && rr_env[0] == '1';
  for (int s0 = 0, c = 0; s0 < TS && !packed; ++c) {
    const bool head = TS - s0 > 16 * chunk;
    int len = (round_robin || head) ? chunk : std::min(chunk, tail_chunk);
    if (head && !round_robin && align_on) {
      // whole problems per chunk: split the rest of this problem's run into near-equal chunks of
      // about `chunk` tiles (a 33-tile expert stays on one XCD instead of spilling 1 tile onto
      // another that re-fetches its A rows), at most 64
      const int rem = seq_end[s0] - s0, nc = std::max(1, (rem + chunk / 2) / chunk);
      len = std::min(64, (rem + nc - 1) / nc);
    }
    const int s1 = std::min(TS, s0 + len);
    // (a chunk can be a whole XCD's slots: 96 for the 3-WG/CU kernel — sized per chunk, not fixed)
    std::vector<double> times(std::max(0, s1 - s0));
    for (int s = s0; s < s1; ++s) times[s - s0] = tile_time(seq[s]);
    int best = c % 8;
    if (!round_robin && head) {  // full chunks: least total time (cheap; the tail evens out)
      best = 0;
      for (int x = 1; x < 8; ++x)
        if (sim[x].load < sim[best].load) best = x;
    } else if (!round_robin) {  // tail: least simulated finish
      double best_finish = 0, best_load = 0;
      for (int x = 0; x < 8; ++x) {
        XcdSim trial = sim[x];
        for (int s = s0; s < s1; ++s) trial.add(times[s - s0]);
        if (x == 0 || trial.finish < best_finish || (trial.finish == best_finish && trial.load < best_load)) {
          best = x;
          best_finish = trial.finish;
          best_load = trial.load;
        }
      }
    }
    for (int s = s0; s < s1; ++s) {
      sim[best].add(times[s - s0]);
      queue[best].push_back(s);
    }
    s0 = s1;
  }
  if (regions_last && !packed) put_regions();

#ifdef MXMOE_LAB
  // Tail split (v2, not persistent). An XCD hands its blocks to its CUs in queue order, so the
  // queue's last tiles run while most of the XCD's CUs have gone idle for good (w8a8 down at
  // bs=8192: 194 tiles per XCD = 6 rounds of 32 + 2; tile timelines put the ragged finish at
  // 6-8 % of CU time). Per XCD, the tiles that start after the first CU's last tile ended are cut
  // along K into S consecutive slices (the split-K path above), S in 2..8 (>= 3 stages a slice,
  // each slice priced at 2 extra stages for its fill and partial-sum traffic) chosen to minimise
  // the XCD's simulated finish; kept only if that gains >= 1 %.
  // MEASURED NEGATIVE: 1.5-2 % slower on the w8a8 / fp16 / mixed gate_up calls, the
  // only layer-11 calls it cuts (the partial-sum round trip costs more than the ragged finish
  // it removes). Lab library only, opt-in: MXMOE_GG_TAIL_SPLIT=1.
  const char* ts_env = planner_knob("MXMOE_GG_TAIL_SPLIT");
  if (v.kind == Kind::V2 && !v.persistent && ts_env && (ts_env[0] == '1' || ts_env[0] == '2')) {
    auto simulate = [&](const std::vector<double>& t, std::vector<double>* starts) {
      std::vector<double> slot(chunk, 0.0);  // min-heap of slot free times
      double finish = 0;
      for (size_t j = 0; j < t.size(); ++j) {
        std::pop_heap(slot.begin(), slot.end(), std::greater<double>());
        if (starts) (*starts)[j] = slot.back();
        slot.back() += t[j];
        finish = std::max(finish, slot.back());
        std::push_heap(slot.begin(), slot.end(), std::greater<double>());
      }
      return std::make_pair(finish, *std::min_element(slot.begin(), slot.end()));
    };
    for (int x = 0; x < 8; ++x) {
      std::vector<int>& q = queue[x];
      const size_t n = q.size();
      if (n <= (size_t)chunk) continue;  // one round: nothing runs after a CU went idle
      std::vector<double> t(n), st(n);
      for (size_t j = 0; j < n; ++j) t[j] = tile_time(all_tiles[q[j]]);
      const auto base = simulate(t, &st);
      size_t j0 = n;
      while (j0 > 0 && st[j0 - 1] >= base.second) --j0;  // starts are non-decreasing in queue order
      auto splittable = [&](const TileDesc& td) {
        const int qt = plan->meta[td.prob].qtype;
        // ('2': weight-only tiles too — the small-batch wo3 calls run ~1.3 rounds of equal tiles)
        return ((td.cls >> 16) & 0xFF) <= 1 && (!is_weightonly(qt) || ts_env[0] == '2') && qt != QT_I4G &&
               td.ks1 - td.ks0 >= 6;
      };
      int best_s = 1;
      double best_finish = base.first;
      for (int S = 2; S <= 8; ++S) {
        std::vector<double> t2(t.begin(), t.begin() + j0);
        for (size_t j = j0; j < n; ++j) {
          const TileDesc& td = all_tiles[q[j]];
          const int nst = td.ks1 - td.ks0;
          if (!splittable(td) || nst / S < 3) {
            t2.push_back(t[j]);
            continue;
          }
          const double per_stage = t[j] / nst;
          for (int k = 0; k < S; ++k) t2.push_back(per_stage * ((k + 1) * nst / S - k * nst / S + 2));
        }
        const double f = simulate(t2, nullptr).first;
        if (f < best_finish) {
          best_finish = f;
          best_s = S;
        }
      }
      if (best_s == 1 || best_finish > 0.99 * base.first) continue;
      std::vector<int> q2(q.begin(), q.begin() + j0);
      for (size_t j = j0; j < n; ++j) {
        const TileDesc td = all_tiles[q[j]];
        const int nst = td.ks1 - td.ks0, S = best_s;
        if (!splittable(td) || nst / S < 3) {
          q2.push_back(q[j]);
          continue;
        }
        const int grp = groups++, slab = plan->slabs;
        plan->slabs += S;
        plan->tail_slabs += S;
        for (int k = 0; k < S; ++k) {
          q2.push_back((int)all_tiles.size());
          all_tiles.push_back(TileDesc{td.prob, td.m0, td.n0, (td.cls & 0xFF) | (k << 8) | (S << 16),
                                       td.ks0 + k * nst / S, td.ks0 + (k + 1) * nst / S, slab, grp});
        }
      }
      q.swap(q2);
    }
  }
#endif
#ifdef MXMOE_LAB
  // Mixed residency (lab A/B, MXMOE_GG_MIX = 1): each XCD queue interleaved so a
  // CU's co-resident workgroups (wo3: three) hold one full-height tile (a shared-expert tile, MFMA-
  // heavy) beside the routed tiles of ~35 rows (weight-stream-heavy) instead of all-shared, then
  // all-routed rounds: the routed tiles' stream then runs under the shared tiles' MFMAs. "Full" =
  // a tile whose modelled time is at least 1.3x the queue's median.
  const char* mix_env = planner_knob("MXMOE_GG_MIX");
  if (mix_env && mix_env[0] == '1' && v.kind == Kind::V2 && !v.persistent) {
    for (auto& q : queue) {
      if (q.size() < 4) continue;
      std::vector<double> t(q.size());
      for (size_t j = 0; j < q.size(); ++j) t[j] = tile_time(all_tiles[q[j]]);
      std::vector<double> srt(t);
      std::nth_element(srt.begin(), srt.begin() + srt.size() / 2, srt.end());
      const double med = srt[srt.size() / 2];
      std::vector<int> lo, hi;
      for (size_t j = 0; j < q.size(); ++j) ((t[j] >= 1.3 * med) ? hi : lo).push_back(q[j]);
      if (hi.empty() || lo.empty()) continue;
      std::vector<int> out;
      size_t a = 0, b = 0;
      while (a < hi.size() || b < lo.size()) {  // keep the hi : lo proportion along the queue
        if (b >= lo.size() || (a < hi.size() && a * lo.size() <= b * hi.size())) out.push_back(hi[a++]);
        else out.push_back(lo[b++]);
      }
      q.swap(out);
    }
  }
#endif
  size_t qmax = 0;
  for (const auto& q : queue) qmax = std::max(qmax, q.size());
  int grid = 0;
  plan->tiles.assign(8 * qmax, TileDesc{-1, 0, 0, 0, 0, 0, -1, -1});
  for (int x = 0; x < 8; ++x)
    for (size_t i = 0; i < queue[x].size(); ++i) {
      const int b = (int)(8 * i) + x;
      plan->tiles[b] = all_tiles[queue[x][i]];
      grid = std::max(grid, b + 1);
    }
  plan->tiles.resize(grid);
  plan->total_tiles = 0;
  for (const auto& q : queue) plan->total_tiles += (int)q.size();
#ifdef MXMOE_LAB
  // Low-fill LPT (lab opt-in, MXMOE_GG_LOWFILL_LPT=1): a call of at most 4 tiles per CU is laid out
  // as one list in descending modelled tile time (stable: a tile's split-K slices and a band's
  // m-tiles stay adjacent); block b then lands on XCD b % 8 and each XCD hands its sublist to its
  // CUs in LPT order. At 2-3 tiles per CU the XCD chunks above concentrate the long tiles (the
  // shared expert's split slices) on 2-3 XCDs, and the tile traces show 15-36 % ragged finish.
  const char* lpt_env = planner_knob("MXMOE_GG_LOWFILL_LPT");
  if (lpt_env && lpt_env[0] == '1' && v.kind == Kind::V2 && !v.persistent && plan->total_tiles <= 4 * 8 * chunk) {
    std::vector<TileDesc> list;
    for (const TileDesc& td : plan->tiles)
      if (td.prob >= 0) list.push_back(td);
    std::stable_sort(list.begin(), list.end(),
                     [&](const TileDesc& a, const TileDesc& b) { return tile_time(a) > tile_time(b); });
    plan->tiles = list;
    grid = (int)list.size();
  }
#endif
  plan->launch_grid = grid;
  if (v.persistent && v.persist_len > 0) {
    // v2q with block lists: XCD x's queue cut into groups of L consecutive tiles, group g run by
    // block 8 g + x (that XCD under round-robin placement: speed only); the hardware hands a freed
    // CU the next block, as for the one-tile blocks. Table [k][G] with a terminating row.
    const int L = v.persist_len;
    size_t ngroups = 0;
    for (const auto& q : queue) ngroups = std::max(ngroups, (q.size() + L - 1) / L);
    const int G = (int)(8 * ngroups);
    plan->tiles.assign((size_t)(L + 1) * G, TileDesc{-1, 0, 0, 0, 0, 0, -1, -1});
    for (int x = 0; x < 8; ++x)
      for (size_t j = 0; j < queue[x].size(); ++j) {
        const size_t g = j / L, k = j % L;
        plan->tiles[k * G + 8 * g + x] = all_tiles[queue[x][j]];
      }
    plan->launch_grid = T > 0 ? G : 0;
  } else if (v.persistent) {
    // v2p: each XCD's queue handed out to its `chunk` workgroups in queue order, every tile to the
    // workgroup whose modelled finish is earliest (what the hardware's dispatch does with blocks,
    // planned once here); workgroup w = 8 * slot + x sits on XCD x under round-robin placement
    // (speed only). Table [k][G] with a terminating row of empty slots.
    const int G = 8 * chunk;
    std::vector<std::vector<int>> lists(G);
    for (int x = 0; x < 8; ++x) {
      std::vector<std::pair<double, int>> heap;
      for (int sl = 0; sl < chunk; ++sl) heap.push_back({0.0, sl});
      std::make_heap(heap.begin(), heap.end(), std::greater<std::pair<double, int>>());
      for (int idx : queue[x]) {
        std::pop_heap(heap.begin(), heap.end(), std::greater<std::pair<double, int>>());
        auto& top = heap.back();
        lists[8 * top.second + x].push_back(idx);
        top.first += tile_time(all_tiles[idx]);
        std::push_heap(heap.begin(), heap.end(), std::greater<std::pair<double, int>>());
      }
    }
    size_t maxlen = 0;
    for (const auto& l : lists) maxlen = std::max(maxlen, l.size());
    plan->tiles.assign((maxlen + 1) * G, TileDesc{-1, 0, 0, 0, 0, 0, -1, -1});
    for (int w = 0; w < G; ++w)
      for (size_t k = 0; k < lists[w].size(); ++k) plan->tiles[k * G + w] = all_tiles[lists[w][k]];
    plan->launch_grid = T > 0 ? G : 0;
  }
  return MXMOE_GG_OK;
}

int check_variant(int variant) {
  if (variant < 0 || variant >= (int)variants().size())
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "variant %d not compiled (have %d)", variant, (int)variants().size());
  return MXMOE_GG_OK;
}

// MXMOE_GG_VARIANT_AUTO -> concrete variant from the quant types present (policy above).
int resolve_variant(int variant, const std::vector<HostProblem>& hp, int* out) {
  if (variant != MXMOE_GG_VARIANT_AUTO) {
    *out = variant;
    return check_variant(variant);
  }
  int mask = 0;
  for (const HostProblem& p : hp) {
    int qt;
    if (p.M > 0 && qtype_of(p.a_bits, p.w_bits, p.gsize, p.sym, p.fmt, &qt) == MXMOE_GG_OK) mask |= 1 << qt;
  }
  *out = variant_index(kDefaultVariantName);
  const int wo_mask = (1 << QT_W4A16) | (1 << QT_W8A16) | (1 << QT_W2A16);
  const int small_mask = wo_mask | (1 << QT_I8) | (1 << QT_F16) | (1 << QT_I4);
  // (fused SiLU calls too: the small-batch kernel's fp16 / w8a8 / w4a4 bodies carry the epilogue)
  if (mask != 0 && (mask & ~small_mask) == 0) {
    // (w8a8 / fp16 problems may ride along: the reference's small-batch w4a16 + w8a8 pairing)
    double wsum0 = 0, ksum = 0;
    int kmax = 0;
    for (const HostProblem& p : hp) {
      if (p.M <= 0 || p.N <= 0) continue;
      const double w = (double)p.N * p.K;
      wsum0 += w;
      ksum += w * p.K;
      kmax = std::max(kmax, p.K);
    }
    const bool kskew = wsum0 > 0 && kmax >= 2.0 * ksum / wsum0;
    const double limit = (mask & wo_mask) ? kWoSmallMeanRows
                                          : ((mask & (1 << QT_I4)) ? kSmallMeanRowsI4 : kSmallMeanRows) * (kskew ? 2.0 : 1.0);
    // weight-only: the 3-WG/CU 64-row kernel while the rows per weight byte are few (small batches:
    // the 64-row tile is bound by its instruction stream and barriers, a second and third resident
    // workgroup fill each other's waits — +15-70 % on the qwen2_moe calls at bs 128-2048,
    // profiles/r03/wo2/); v2x's 256-row tiles at large batch
    double wsum = 0, msum = 0;
    for (const HostProblem& p : hp) {
      if (p.M <= 0 || p.N <= 0) continue;
      const double w = (double)p.N * p.K;
      wsum += w;
      msum += w * p.M;
    }
    if (wsum > 0 && msum / wsum <= limit) {
      const int wi = variant_index(kWoSmallVariant);
      if (!strcmp(variants()[wi].name, kWoSmallVariant)) {
        *out = wi;
        return MXMOE_GG_OK;
      }
    }
  }
#ifdef MXMOE_LAB
  if ((mask & (1 << QT_I4F6)) && mask != (1 << QT_I4F6))
    return fail(MXMOE_GG_ERR_UNSUPPORTED,
                "fp6-image w4a4 problems (MXMOE_GG_FMT_F6) cannot share a call with other quant types: plan them "
                "as a call of their own");
  if (mask == (1 << QT_I4F6)) {  // fp6 images: the fp6 kernel (no other variant reads them)
    *out = variant_index(kF6Variant);
    return MXMOE_GG_OK;
  }
#endif
  if (mask == (1 << QT_I4)) {
    // int4-only: the 256x128 2-WG/CU kernel, unless the call is low-fill enough for the v2s plan
    // to split K (that kernel cannot)
    Plan p;
    if (plan_host(hp, *out, false, &p) == MXMOE_GG_OK && p.slabs == p.tail_slabs) *out = variant_index(kInt4Variant);
  }
  return MXMOE_GG_OK;
}

std::vector<HostProblem> to_host(const mxmoe_gg_problem* problems, int problem_count) {
  std::vector<HostProblem> hp(problem_count);
  for (int i = 0; i < problem_count; ++i) {
    const mxmoe_gg_problem& p = problems[i];
    hp[i] = HostProblem{p.A,      p.B,      p.scale_a, p.scale_b, p.C,   p.M,   p.N,  p.K,
                        p.a_bits, p.w_bits, p.gsize,   p.sym,     p.lda, p.ldb, p.ldc, p.fmt};
  }
  return hp;
}

// Host image of the workspace for a plan; pointer columns from `hp` in table-row order.
std::vector<uint8_t> workspace_image(const Plan& plan, const std::vector<const void*> cols[5], WsLayout* out) {
  const int P = (int)plan.meta.size();
  const WsLayout l = ws_layout(P, (int)plan.tiles.size(), plan.slabs);
  std::vector<uint8_t> img(l.total - l.slabs, 0);  // counters start at zero; slabs need no init
  memcpy(img.data(), plan.meta.data(), (size_t)P * sizeof(GGMeta));
  for (int c = 0; c < 5; ++c) memcpy(img.data() + l.meta + c * l.ptr, cols[c].data(), (size_t)P * sizeof(void*));
  memcpy(img.data() + l.meta + 5 * l.ptr, plan.tiles.data(), plan.tiles.size() * sizeof(TileDesc));
  *out = l;
  return img;
}

// FNV-1a over the plan table and the tile table: equal for two calls with the same shapes, quant
// params and strides (the planner is deterministic), whatever their buffers.
uint64_t plan_signature(const Plan& plan) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  };
  mix(plan.meta.data(), plan.meta.size() * sizeof(GGMeta));
  mix(plan.tiles.data(), plan.tiles.size() * sizeof(TileDesc));
  mix(plan.order.data(), plan.order.size() * sizeof(int));
  return h;
}

void fill_info(const Plan& plan, int variant, const WsLayout& l, void* ws, mxmoe_gg_plan_info* info) {
  const Variant& v = variants()[variant];
  info->variant = variant;
  info->problem_count = (int)plan.meta.size();
  info->total_tiles = plan.total_tiles;
  info->grid = plan.launch_grid;
  info->tile_slots = (int)plan.tiles.size();
  info->reserved = 0;
  info->block = v.threads;
  info->qtype_mask = 0;
  for (const GGMeta& m : plan.meta) {
    info->qtype_mask |= 1 << m.qtype;
    if (is_weightonly(m.qtype) && (m.reserved2 & META_SILU)) info->qtype_mask |= kQmaskWoSilu;
  }
  info->lds_bytes = v.lds_of ? v.lds_of(info->qtype_mask) : v.lds_bytes;
  info->splitk_slabs = plan.slabs;
  info->workspace_bytes = (int64_t)l.total;
  info->workspace = ws;
  info->signature = plan_signature(plan);
}

}  // namespace

namespace mxmoe {
namespace detail {
// error channel shared with the MoE plumbing (moe_ops.hip)
int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
}  // namespace detail
}  // namespace mxmoe

extern "C" {

int mxmoe_gg_abi_version(void) { return MXMOE_GG_ABI_VERSION; }

const char* mxmoe_gg_last_error(void) { return g_last_error.c_str(); }

int mxmoe_gg_variant_count(void) { return (int)variants().size(); }

int mxmoe_gg_default_variant(void) { return variant_index(kDefaultVariantName); }

int mxmoe_gg_list_variants(char* buf, size_t n) {
  // weight-only kernels cover every group size / sym of a bit width: listed under the base name
  static const char* qnames[QT_COUNT] = {"fp16",          "w8a8_g-1_sym", "w4a4_g-1_sym",      "w4a16", "w8a16",
                                         "w4a4_g128_sym", "w2a16",        "w8a8_g-1_sym_E4M3", "bf16",  "w4a4_g-1_sym_F6"};
  static const int wbits[QT_COUNT] = {16, 8, 4, 4, 8, 4, 2, 8, 16, 6};
  std::string out;
  const auto& vs = variants();
  for (size_t i = 0; i < vs.size(); ++i) {
    char line[1024];
    int off = snprintf(line, sizeof(line), "%zu %s", i, vs[i].name);
    for (int q = 0; q < QT_COUNT; ++q) {
      const TileGeom& g = vs[i].geom[q];
      if (g.bn == 0) continue;  // quant type not implemented by this variant
      const int bits = wbits[q];
      const int waves = g.threads / 64;
      const int wm = 2, wn = waves / wm;
      off += snprintf(line + off, sizeof(line) - off,
                      " %s=TileConfig(BM=%d, BN=%d, BK=%d, WM=%d, WN=%d, WK=1, STAGE=2)", qnames[q], g.bm, g.bn,
                      g.bkb * 8 / bits, wm, wn);
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

int mxmoe_gg_variant_caps(int variant, uint32_t* caps) {
  if (!caps) return fail(MXMOE_GG_ERR_INVALID, "caps is NULL");
  if (int st = check_variant(variant)) return st;
  *caps = has_silu_epilogue(variants()[variant]) ? MXMOE_GG_CAP_SILU_MUL : 0u;
  return MXMOE_GG_OK;
}

int mxmoe_gg_variant_tile(int variant, int a_bits, int w_bits, int32_t* bm, int32_t* bn, int32_t* bk_bytes,
                          int32_t* threads) {
  int st = check_variant(variant);
  if (st) return st;
  int qt = 0;
  st = qtype_of(a_bits, w_bits, -1, 1, MXMOE_GG_FMT_DEFAULT, &qt);
  if (st) return st;
  const TileGeom& g = variants()[variant].geom[qt];
  if (bm) *bm = g.bm;
  if (bn) *bn = g.bn;
  if (bk_bytes) *bk_bytes = g.bkb;
  if (threads) *threads = g.threads;
  return MXMOE_GG_OK;
}

#ifdef MXMOE_LAB
// lab-only exports (tools/f6_bench.py, tests/test_f6.py): int4 rows -> fp6 images (gg_f6.h layout)
namespace {
int f6_args(const void* src, int rows, int K, int64_t ld_src, const void* dst, int64_t ld_dst, int64_t* ls, int64_t* ld) {
  if (rows < 0 || K < 0 || (rows > 0 && (!src || !dst))) return fail(MXMOE_GG_ERR_INVALID, "pack_f6: bad arguments");
  if (K % 32) return fail(MXMOE_GG_ERR_INVALID, "pack_f6: K=%d must be a multiple of 32 (16-B int4 rows)", K);
  *ls = ld_src ? ld_src * 2 : K / 2;
  *ld = ld_dst ? ld_dst * 2 : MXMOE_GG_F6_ROW_BYTES(K);
  if (*ls < K / 2 || *ld < MXMOE_GG_F6_ROW_BYTES(K) || (*ls % 16) || (*ld % 16))
    return fail(MXMOE_GG_ERR_INVALID, "pack_f6: row strides must cover the row and be multiples of 8 words");
  if (rows > 0 && (((uintptr_t)src | (uintptr_t)dst) & 15))
    return fail(MXMOE_GG_ERR_INVALID, "pack_f6: buffers must be 16-B aligned");
  return MXMOE_GG_OK;
}
}  // namespace

int mxmoe_gg_pack_f6(const void* src, int rows, int K, int64_t ld_src, void* dst, int64_t ld_dst, void* stream) {
  int64_t ls, ld;
  int st = f6_args(src, rows, K, ld_src, dst, ld_dst, &ls, &ld);
  if (st) return st;
  const int64_t threads = (int64_t)rows * ((K + 127) / 128) * 4;
  if (threads == 0) return MXMOE_GG_OK;
  hipLaunchKernelGGL(f6_pack_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const uint8_t*>(src), ls, static_cast<uint8_t*>(dst), ld, rows, K);
  HIP_TRY(hipGetLastError());
  return MXMOE_GG_OK;
}

int mxmoe_gg_pack_f6_host(const void* src, int rows, int K, int64_t ld_src, void* dst, int64_t ld_dst) {
  int64_t ls, ld;
  int st = f6_args(src, rows, K, ld_src, dst, ld_dst, &ls, &ld);
  if (st) return st;
  const int nblk = (K + 127) / 128;
  for (int64_t r = 0; r < rows; ++r)
    for (int b = 0; b < nblk; ++b)
      for (int g = 0; g < 4; ++g) {
        const int e0 = b * 128 + g * 32;
        uint32_t w[4] = {0, 0, 0, 0};
        if (e0 < K) memcpy(w, static_cast<const uint8_t*>(src) + r * ls + e0 / 2, 16);  // (K % 32 == 0)
        uint32_t d[6];
        f6_pack32(w, d);
        uint8_t* o = static_cast<uint8_t*>(dst) + r * ld + b * 96;
        memcpy(o + g * 16, d, 16);
        memcpy(o + 64 + g * 8, d + 4, 8);
      }
  return MXMOE_GG_OK;
}
#endif  // MXMOE_LAB

int mxmoe_gg_resolve_variant(const mxmoe_gg_problem* problems, int problem_count, int variant, int* out) {
  if (!out) return fail(MXMOE_GG_ERR_INVALID, "out is NULL");
  if (problem_count < 0 || (problem_count > 0 && !problems))
    return fail(MXMOE_GG_ERR_INVALID, "bad problem array (count %d)", problem_count);
  return resolve_variant(variant, to_host(problems, problem_count), out);
}

int mxmoe_gg_workspace_size(const mxmoe_gg_problem* problems, int problem_count, int variant, size_t* bytes) {
  if (problem_count < 0 || (problem_count > 0 && !problems) || !bytes)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_workspace_size");
  const std::vector<HostProblem> hp = to_host(problems, problem_count);
  int st = resolve_variant(variant, hp, &variant);
  if (st) return st;
  Plan plan;
  st = plan_host(hp, variant, false, &plan);
  if (st) return st;
  *bytes = ws_layout((int)plan.meta.size(), (int)plan.tiles.size(), plan.slabs).total;
  return MXMOE_GG_OK;
}

int mxmoe_gg_plan_tiles(const mxmoe_gg_problem* problems, int problem_count, int variant, int32_t* tiles,
                        int32_t* rows, int* slots) {
  if (problem_count < 0 || (problem_count > 0 && !problems) || !slots || *slots < 0 || (*slots > 0 && !tiles))
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_plan_tiles");
  const std::vector<HostProblem> hp = to_host(problems, problem_count);
  int st = resolve_variant(variant, hp, &variant);
  if (st) return st;
  Plan plan;
  st = plan_host(hp, variant, false, &plan);
  if (st) return st;
  const int n = std::min(*slots, (int)plan.tiles.size());
  if (n > 0) memcpy(tiles, plan.tiles.data(), (size_t)n * sizeof(TileDesc));
  if (rows)
    for (size_t r = 0; r < plan.order.size(); ++r) rows[r] = plan.order[r];
  *slots = (int)plan.tiles.size();
  return MXMOE_GG_OK;
}

// What mxmoe_gg_rebind needs of a plan to skip the host planner: per workspace, a key over
// everything plan_host reads except the pointers, the plan's signature and its table-row order.
// A later mxmoe_gg_plan into the same workspace replaces the entry.
struct RebindEntry {
  uint64_t key = 0, signature = 0;
  std::vector<int> order;
};
static std::mutex g_rebind_mu;
static std::unordered_map<const void*, RebindEntry> g_rebind;
static uint64_t rebind_key(const std::vector<HostProblem>& hp, int variant) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)variant;
  auto mix = [&](int64_t v) {
    h ^= (uint64_t)v;
    h *= 1099511628211ull;
  };
  mix((int64_t)hp.size());
  for (const HostProblem& p : hp)
    for (int64_t v : {(int64_t)p.M, (int64_t)p.N, (int64_t)p.K, (int64_t)p.a_bits, (int64_t)p.w_bits, (int64_t)p.gsize,
                      (int64_t)p.sym, (int64_t)p.fmt, p.lda, p.ldb, p.ldc})
      mix(v);
  return h;
}
// Invariant: every plan written into a workspace goes through mxmoe_gg_plan, which calls
// remember_plan and so replaces the workspace's entry. An entry outlives its workspace only as a
// stale key: a new workspace at the same address is planned (and re-remembered) before any rebind,
// and mxmoe_gg_forget_workspace drops the entry when the caller frees the buffer.
static void remember_plan(const void* ws, const std::vector<HostProblem>& hp, int variant, const Plan& plan) {
  std::lock_guard<std::mutex> lk(g_rebind_mu);
  if (g_rebind.size() >= 1024 && !g_rebind.count(ws)) g_rebind.clear();
  RebindEntry& e = g_rebind[ws];
  e.key = rebind_key(hp, variant);
  e.signature = plan_signature(plan);
  e.order = plan.order;
}

int mxmoe_gg_plan(const mxmoe_gg_problem* problems, int problem_count, int variant, void* workspace,
                  size_t workspace_bytes, void* stream, mxmoe_gg_plan_info* info) {
  if (problem_count < 0 || (problem_count > 0 && !problems) || !info)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_plan");
  const std::vector<HostProblem> hp = to_host(problems, problem_count);
  int st = resolve_variant(variant, hp, &variant);
  if (st) return st;
  Plan plan;
  st = plan_host(hp, variant, true, &plan);
  if (st) return st;
  std::vector<const void*> cols[5];
  for (int r : plan.order) {
    cols[0].push_back(hp[r].A);
    cols[1].push_back(hp[r].B);
    cols[2].push_back(hp[r].SA);
    cols[3].push_back(hp[r].SB);
    cols[4].push_back(hp[r].C);
  }
  WsLayout l;
  std::vector<uint8_t> img = workspace_image(plan, cols, &l);
  if (!workspace || workspace_bytes < l.total)
    return fail(MXMOE_GG_ERR_WORKSPACE, "workspace too small: need %zu bytes, have %zu", l.total, workspace_bytes);
  HIP_TRY(hipMemcpyAsync(workspace, img.data(), img.size(), hipMemcpyHostToDevice, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // pageable host image must outlive the copy
  fill_info(plan, variant, l, workspace, info);
  remember_plan(workspace, hp, variant, plan);
  return MXMOE_GG_OK;
}

int mxmoe_gg_forget_workspace(const void* workspace) {
  std::lock_guard<std::mutex> lk(g_rebind_mu);
  g_rebind.erase(workspace);
  return MXMOE_GG_OK;
}

int mxmoe_gg_rebind(const mxmoe_gg_problem* problems, int problem_count, const mxmoe_gg_plan_info* info,
                    void* stream) {
  if (problem_count < 0 || (problem_count > 0 && !problems) || !info || !info->workspace)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_rebind");
  int st = check_variant(info->variant);
  if (st) return st;
  const std::vector<HostProblem> hp = to_host(problems, problem_count);
  // fast path: the same shapes / quant params / strides as this workspace's plan -> only the
  // pointers are checked (build_meta's NULL / alignment checks), the tile planner is skipped
  // (only a real key + signature hit takes it: an all-empty plan has an empty order too, and rebinding
  // it with non-empty problems must go through the planner and fail the signature check)
  std::vector<int> order;
  bool hit = false;
  {
    const uint64_t key = rebind_key(hp, info->variant);
    std::lock_guard<std::mutex> lk(g_rebind_mu);
    auto it = g_rebind.find(info->workspace);
    if (it != g_rebind.end() && it->second.key == key && it->second.signature == info->signature) {
      order = it->second.order;
      hit = true;
    }
  }
  if (hit) {
    const Variant& v = variants()[info->variant];
    for (int i = 0; i < (int)hp.size(); ++i) {
      GGMeta m;
      st = build_meta(hp[i], i, v, true, &m);
      if (st) return st;
    }
  } else {
    Plan plan;
    st = plan_host(hp, info->variant, true, &plan);
    if (st) return st;
    if (plan_signature(plan) != info->signature || (int)plan.meta.size() != info->problem_count)
      return fail(MXMOE_GG_ERR_INVALID, "mxmoe_gg_rebind: problems differ from the planned call (shapes, quant "
                                        "params or strides); plan again");
    order = plan.order;
  }
  if ((int)order.size() != info->problem_count)
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_gg_rebind: problems differ from the planned call; plan again");
  const WsLayout l = ws_layout(info->problem_count, info->tile_slots, info->splitk_slabs);
  std::vector<uint8_t> cols(5 * l.ptr, 0);
  for (int c = 0; c < 5; ++c)
    for (size_t i = 0; i < order.size(); ++i) {
      const HostProblem& q = hp[order[i]];
      const void* p = c == 0 ? q.A : c == 1 ? q.B : c == 2 ? q.SA : c == 3 ? q.SB : q.C;
      memcpy(cols.data() + c * l.ptr + i * sizeof(void*), &p, sizeof(void*));
    }
  HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(info->workspace) + l.meta, cols.data(), cols.size(),
                         hipMemcpyHostToDevice, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));  // pageable host columns must outlive the copy
  return MXMOE_GG_OK;
}

int mxmoe_gg_launch(const mxmoe_gg_plan_info* info, void* stream) {
  if (!info) return fail(MXMOE_GG_ERR_INVALID, "NULL plan");
  int st = check_variant(info->variant);
  if (st) return st;
  if (info->total_tiles == 0) return MXMOE_GG_OK;
  const int P = info->problem_count;
  const WsLayout l = ws_layout(P, info->tile_slots, info->splitk_slabs);
  const uint8_t* ws = static_cast<const uint8_t*>(info->workspace);
  GGArgs a;
  a.meta = reinterpret_cast<const GGMeta*>(ws);
  a.tiles = reinterpret_cast<const TileDesc*>(ws + l.meta + 5 * l.ptr);
  a.ptr_A = reinterpret_cast<const void* const*>(ws + l.meta);
  a.ptr_B = reinterpret_cast<const void* const*>(ws + l.meta + l.ptr);
  a.ptr_SA = reinterpret_cast<const void* const*>(ws + l.meta + 2 * l.ptr);
  a.ptr_SB = reinterpret_cast<const void* const*>(ws + l.meta + 3 * l.ptr);
  a.ptr_C = reinterpret_cast<void* const*>(ws + l.meta + 4 * l.ptr);
  a.P = P;
  a.n_slots = info->grid;
  a.counters = reinterpret_cast<int32_t*>(const_cast<uint8_t*>(ws) + l.meta + 5 * l.ptr + l.tiles);
  a.slabs = const_cast<uint8_t*>(ws) + l.meta + 5 * l.ptr + l.tiles + l.counters;
  variants()[info->variant].launch(a, info->grid, info->qtype_mask, (hipStream_t)stream);
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

// Reference-compatible entry point (registry.cuh:28-39): device pointer arrays, host copies of
// the sizes and QParams, legacy default stream, per-call planning (as the reference host API).
// Per-device resources of the reference-ABI shim (the only entry that allocates): a device
// workspace grown on demand and a pinned host staging buffer for the pointer gather and the
// workspace image. Keyed by the calling thread's current device; one mutex per process guards the
// table and serialises shim calls (the reference's host API is not reentrant either, it runs
// cudaMalloc / cudaMemcpy / cudaFree on the legacy stream every call, kernel_sketch.py:102-143).
namespace {
struct ShimDev {
  void* ws = nullptr;
  size_t ws_cap = 0;
  uint8_t* pinned = nullptr;
  size_t pin_cap = 0;
  // plan cache: the last call's shapes / quant params (key), its plan, and the pointer columns the
  // workspace holds. A call with the same key skips planning and the tile-table upload (a caller
  // runs the same layer shapes call after call); new pointers re-upload the columns only.
  bool cached = false;
  std::vector<int64_t> key;
  Plan plan;
  int variant = -1;
  WsLayout layout{};
  std::vector<const void*> cols;  // 5 x P, plan order, as in the workspace
};
std::mutex g_shim_mu;
std::vector<ShimDev> g_shim;  // indexed by device ordinal

int shim_grow(ShimDev& d, size_t ws_bytes, size_t pin_bytes) {
  if ((d.ws_cap < ws_bytes && d.ws) || (d.pin_cap < pin_bytes && d.pinned))
    HIP_TRY(hipStreamSynchronize(nullptr));  // a previous shim copy / launch may still use the old buffer
  if (d.ws_cap < ws_bytes) {
    if (d.ws) HIP_TRY(hipFree(d.ws));
    d.ws = nullptr;
    d.ws_cap = 0;
    HIP_TRY(hipMalloc(&d.ws, ws_bytes));
    d.ws_cap = ws_bytes;
  }
  if (d.pin_cap < pin_bytes) {
    if (d.pinned) HIP_TRY(hipHostFree(d.pinned));
    d.pinned = nullptr;
    d.pin_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&d.pinned, pin_bytes, hipHostMallocDefault));
    d.pin_cap = pin_bytes;
  }
  return MXMOE_GG_OK;
}
}  // namespace

int mxmoe_gg_release_shim_workspaces(void) {
  std::lock_guard<std::mutex> lk(g_shim_mu);
  int dev0 = 0;
  HIP_TRY(hipGetDevice(&dev0));
  for (size_t i = 0; i < g_shim.size(); ++i) {
    ShimDev& d = g_shim[i];
    if (!d.ws && !d.pinned) continue;
    HIP_TRY(hipSetDevice((int)i));
    HIP_TRY(hipDeviceSynchronize());  // the last shim launch on this device may still read the workspace
    if (d.ws) HIP_TRY(hipFree(d.ws));
    if (d.pinned) HIP_TRY(hipHostFree(d.pinned));
    d = ShimDev{};
  }
  HIP_TRY(hipSetDevice(dev0));
  return MXMOE_GG_OK;
}

int groupgemm_mxmoe(void** ptr_As, void** ptr_Bs, void** ptr_scale_a, void** ptr_scale_b, void** ptr_Cs,
                    void** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                    mxmoe_dim3* problem_sizes, mxmoe_dim3* h_problem_sizes, mxmoe_qparams* qbits_list,
                    mxmoe_qparams* h_qbits_list, int problem_count) {
  return groupgemm_mxmoe_fmt(ptr_As, ptr_Bs, ptr_scale_a, ptr_scale_b, ptr_Cs, ptr_Ds, ldas, ldbs, ldcs, ldds,
                             problem_sizes, h_problem_sizes, qbits_list, h_qbits_list, problem_count, nullptr);
}

int groupgemm_mxmoe_fmt(void** ptr_As, void** ptr_Bs, void** ptr_scale_a, void** ptr_scale_b, void** ptr_Cs,
                        void** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                        mxmoe_dim3* problem_sizes, mxmoe_dim3* h_problem_sizes, mxmoe_qparams* qbits_list,
                        mxmoe_qparams* h_qbits_list, int problem_count, const int32_t* h_fmts) {
  (void)ptr_Ds;
  (void)ldas;
  (void)ldbs;
  (void)ldcs;
  (void)ldds;
  (void)problem_sizes;
  (void)qbits_list;
  if (problem_count < 0 || !h_problem_sizes || !h_qbits_list)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to groupgemm_mxmoe");
  if (problem_count == 0) return MXMOE_GG_OK;
  void** src[5] = {ptr_As, ptr_Bs, ptr_scale_a, ptr_scale_b, ptr_Cs};
  for (int c = 0; c < 5; ++c)
    if (!src[c]) return fail(MXMOE_GG_ERR_INVALID, "groupgemm_mxmoe: NULL device pointer array");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_shim_mu);
  if ((int)g_shim.size() <= dev) g_shim.resize(dev + 1);
  ShimDev& d = g_shim[dev];
  // 1. gather the caller's device pointer arrays: 5 async copies into pinned memory, ONE sync (the
  //    reference pays one blocking cudaMemcpy per call, kernel_sketch.py:102-104)
  const size_t col = (size_t)problem_count * sizeof(void*);
  int st = shim_grow(d, 0, 5 * col);
  if (st) return st;
  for (int c = 0; c < 5; ++c)
    HIP_TRY(hipMemcpyAsync(d.pinned + c * col, src[c], col, hipMemcpyDeviceToHost, nullptr));
  HIP_TRY(hipStreamSynchronize(nullptr));
  void* const* h = reinterpret_cast<void* const*>(d.pinned);
  std::vector<HostProblem> hp(problem_count);
  for (int i = 0; i < problem_count; ++i)
    hp[i] = HostProblem{h[0 * problem_count + i], h[1 * problem_count + i], h[2 * problem_count + i],
                        h[3 * problem_count + i], h[4 * problem_count + i], (int)h_problem_sizes[i].x,
                        (int)h_problem_sizes[i].y, (int)h_problem_sizes[i].z, h_qbits_list[i].a_bits,
                        h_qbits_list[i].w_bits, h_qbits_list[i].gsize, h_qbits_list[i].sym, 0, 0, 0,
                        h_fmts ? (int)h_fmts[i] : (int)MXMOE_GG_FMT_DEFAULT};  // never QParams' padding
  // 2. same shapes as the last call on this device: reuse its plan (the pointers still get the same
  //    NULL / alignment checks as mxmoe_gg_plan)
  std::vector<int64_t> key;
  key.reserve((size_t)problem_count * 8);
  for (const HostProblem& p : hp)
    key.insert(key.end(), {p.M, p.N, p.K, p.a_bits, p.w_bits, p.gsize, p.sym, p.fmt});
  if (d.cached && key == d.key) {
    const Variant& v = variants()[d.variant];
    std::vector<const void*> cols;
    cols.reserve(5 * d.plan.order.size());
    for (int c = 0; c < 5; ++c)
      for (int r : d.plan.order) {
        GGMeta m;
        if (c == 0) {
          st = build_meta(hp[r], r, v, true, &m);
          if (st) return st;
        }
        const HostProblem& q = hp[r];
        cols.push_back(c == 0 ? q.A : c == 1 ? q.B : c == 2 ? q.SA : c == 3 ? q.SB : q.C);
      }
    if (cols != d.cols) {  // new buffers, same shapes: upload the 5 pointer columns only
      const size_t P = d.plan.order.size();
      std::memset(d.pinned, 0, 5 * d.layout.ptr);
      for (int c = 0; c < 5; ++c) memcpy(d.pinned + c * d.layout.ptr, cols.data() + c * P, P * sizeof(void*));
      HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(d.ws) + d.layout.meta, d.pinned, 5 * d.layout.ptr,
                             hipMemcpyHostToDevice, nullptr));
      d.cols = std::move(cols);
    }
    mxmoe_gg_plan_info info;
    fill_info(d.plan, d.variant, d.layout, d.ws, &info);
    return mxmoe_gg_launch(&info, nullptr);
  }
  d.cached = false;
  // 3. plan with the same NULL / alignment checks as mxmoe_gg_plan (a bad pointer is an error code,
  //    never a fault inside the LDS-DMA kernel)
  int variant;
  st = resolve_variant(MXMOE_GG_VARIANT_AUTO, hp, &variant);
  if (st) return st;
  Plan plan;
  st = plan_host(hp, variant, true, &plan);
  if (st) return st;
  if (plan.total_tiles == 0) return MXMOE_GG_OK;
  std::vector<const void*> cols[5];
  for (int r : plan.order) {
    cols[0].push_back(hp[r].A);
    cols[1].push_back(hp[r].B);
    cols[2].push_back(hp[r].SA);
    cols[3].push_back(hp[r].SB);
    cols[4].push_back(hp[r].C);
  }
  WsLayout l;
  std::vector<uint8_t> img = workspace_image(plan, cols, &l);
  // 4. upload from pinned memory and launch, both on the legacy stream, no further host sync: the
  //    next shim call on this device synchronises that stream before it rewrites either buffer
  st = shim_grow(d, l.total, std::max(std::max(5 * col, img.size()), 5 * l.ptr));
  if (st) return st;
  memcpy(d.pinned, img.data(), img.size());
  HIP_TRY(hipMemcpyAsync(d.ws, d.pinned, img.size(), hipMemcpyHostToDevice, nullptr));
  mxmoe_gg_plan_info info;
  fill_info(plan, variant, l, d.ws, &info);
  st = mxmoe_gg_launch(&info, nullptr);
  if (st) return st;
  d.key = std::move(key);
  d.variant = variant;
  d.layout = l;
  d.cols.clear();
  for (int c = 0; c < 5; ++c) d.cols.insert(d.cols.end(), cols[c].begin(), cols[c].end());
  d.plan = std::move(plan);
  d.cached = true;
  return MXMOE_GG_OK;
}


int mxmoe_gg_debug_trace(void* dst, size_t bytes, int reset) {
  const size_t n = std::min(bytes, sizeof(g_gg_trace));
  if (dst && n) HIP_TRY(hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gg_trace), n, 0, hipMemcpyDeviceToHost));
  if (reset) {
    void* p = nullptr;
    HIP_TRY(hipGetSymbolAddress(&p, HIP_SYMBOL(g_gg_trace)));
    HIP_TRY(hipMemset(p, 0, sizeof(g_gg_trace)));
    HIP_TRY(hipDeviceSynchronize());
  }
  return MXMOE_GG_OK;
}

#ifdef MXMOE_LAB
// lab library only (not in include/mxmoe_gg.h): the spread mainloop's per-wave stage stamps
int mxmoe_gg_debug_stamps(void* dst, size_t bytes, int reset) {
  const size_t n = std::min(bytes, sizeof(g_gg_stamp));
  if (dst && n) HIP_TRY(hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gg_stamp), n, 0, hipMemcpyDeviceToHost));
  if (reset) {
    void* p = nullptr;
    HIP_TRY(hipGetSymbolAddress(&p, HIP_SYMBOL(g_gg_stamp)));
    HIP_TRY(hipMemset(p, 0, sizeof(g_gg_stamp)));
    HIP_TRY(hipDeviceSynchronize());
  }
  return MXMOE_GG_OK;
}
#endif

// Inverse of the reference's permute_weight(Row) + pack_weightonly (quantize.cuh:318-421), then
// the kernel layout (include/mxmoe_gg.h). Host code, run once per weight at load time.
int mxmoe_gg_repack_weightonly(const uint16_t* ref_words, int N, int K, int w_bits, uint8_t* out) {
  if (!ref_words || !out || N <= 0 || K <= 0)
    return fail(MXMOE_GG_ERR_INVALID, "bad arguments to mxmoe_gg_repack_weightonly");
  if (w_bits != 2 && w_bits != 4 && w_bits != 8)
    return fail(MXMOE_GG_ERR_UNSUPPORTED, "weight-only repack: w_bits must be 2, 4 or 8 (got %d)", w_bits);
  const int pack = 16 / w_bits, mask = (1 << w_bits) - 1;
  if (N % (pack * 8) || K % 64)
    return fail(MXMOE_GG_ERR_INVALID, "weight-only repack: need N %% %d == 0 and K %% 64 == 0 (N=%d, K=%d)",
                pack * 8, N, K);
  // 1. unpack: word (r, k) holds columns (r/8)*8*pack + f*8 + r%8, f = 0 in the high bits
  std::vector<uint8_t> res((size_t)N * K), orig((size_t)N * K);
  for (int r = 0; r < N / pack; ++r)
    for (int f = 0; f < pack; ++f) {
      const size_t n = (size_t)(r / 8) * 8 * pack + f * 8 + r % 8;
      const int sh = (pack - 1 - f) * w_bits;
      for (int k = 0; k < K; ++k) res[n * K + k] = (uint8_t)((ref_words[(size_t)r * K + k] >> sh) & mask);
    }
  // 2. undo permute_weight: res[idx[x]] = orig[idx[perm[x]]] inside every 16(K) x 8*pack(N) block
  int perm[32];
  {
    const int* proj;
    const int* desired;
    int plen;
    static const int p8[4] = {1, 0, 3, 2}, d8[8] = {0, 2, 4, 6, 1, 3, 5, 7};
    static const int p4[8] = {3, 7, 2, 6, 1, 5, 0, 4};
    static const int d4[16] = {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
    static const int p2[16] = {7, 15, 6, 14, 5, 13, 4, 12, 3, 11, 2, 10, 1, 9, 0, 8};  // quantize.cuh:343-347
    static const int d2[32] = {0, 8,  16, 24, 1, 9,  17, 25, 2, 10, 18, 26, 3, 11, 19, 27,
                               4, 12, 20, 28, 5, 13, 21, 29, 6, 14, 22, 30, 7, 15, 23, 31};
    if (w_bits == 8) {
      proj = p8, desired = d8, plen = 4;
    } else if (w_bits == 4) {
      proj = p4, desired = d4, plen = 8;
    } else {
      proj = p2, desired = d2, plen = 16;
    }
    for (int i = 0; i < 4 * pack; i += plen)
      for (int j = 0; j < plen; ++j) perm[proj[j] + i] = desired[i + j];
  }
  for (int j = 0; j < N; j += pack * 8)
    for (int i = 0; i < K; i += 16)
      for (int tj = 0; tj < 8; ++tj)
        for (int ti = 0; ti < 8; ti += 2) {
          size_t idx[32];
          int x = 0;
          for (int ii = 0; ii < 16; ii += 8)
            for (int tii = 0; tii < 2; ++tii)
              for (int f = 0; f < pack; ++f) idx[x++] = (size_t)(i + ii + ti + tii) + (size_t)(j + f * 8 + tj) * K;
          for (int y = 0; y < x; ++y) orig[idx[perm[y]]] = res[idx[y]];
        }
  // 3. kernel layout
  const size_t row_bytes = (size_t)K * w_bits / 8;
  for (int n = 0; n < N; ++n) {
    uint8_t* o = out + (size_t)n * row_bytes;
    if (w_bits < 8) memset(o, 0, row_bytes);
    for (int k = 0; k < K; ++k) {
      const int seg = k / 64, kl = k % 64, kc = kl / 32, g = (kl % 32) / 8, e = kl % 8;
      // 4-bit: code e of a unit at nibble (e >> 1) | (e & 1) << 2, so codes 2q and 2q+1 are the
      // nibbles at bits 4q and 16 + 4q of the unit's word (one v_and_or_b32 per fp16 pair)
      const int ep = w_bits == 4 ? (e >> 1) | ((e & 1) << 2) : e;
      const size_t pos = (size_t)seg * 64 + g * 16 + kc * 8 + ep;
      const uint8_t u = orig[(size_t)n * K + k];
      if (w_bits == 8) {
        o[pos] = u;
      } else if (w_bits == 4) {
        o[pos / 2] |= (uint8_t)(u << (4 * (pos & 1)));
      } else {
        // 2-bit: the unit (seg, g) is one 32-bit word holding both K halves; code (kc, e) at bit
        // 2 (4 kc + e / 2) for even e and 16 + 2 (4 kc + e / 2) for odd e (fp16 pairs, one and_or)
        const int bit = (e & 1) * 16 + 2 * (4 * kc + e / 2);
        o[(size_t)seg * 16 + g * 4 + bit / 8] |= (uint8_t)(u << (bit % 8));
      }
    }
  }
  return MXMOE_GG_OK;
}

}  // extern "C"
