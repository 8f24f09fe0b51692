// gg_device.h — device side of the MI355X (gfx950) fused mixed-precision GroupGEMM.
//
// What the reference does (SeaCatComplexes/MxMoE, read as text only):
//   persistent fused kernel, per-tile qtype branch ........ compose_kernel.py:150-224, generated/hz_fused_0.cu:12-97
//   tile -> (problem, m-tile, n-tile), n fastest .......... tile_scheduler.cuh:25-50
//   fp16 mainloop (fp32 acc) .............................. cta_gemm.cuh:7-107
//   w8a8 / w4a4 mainloop (exact int32 acc) + epilogue ..... cta_gemm.cuh:423-608
//   epilogue  out = fp16_rn(0 + f32(acc) * f32(fp16_rn(sa*sb))) ... mm_tile.cuh:469-496, 610-662
//
// How it is built here (MI355X-first, not a translation):
//   * one workgroup per output tile, grid = #tiles, XCD-aware bijective blockIdx remap;
//     tile -> problem by binary search over the tile-begin column of the plan table;
//   * K staged 128 BYTES per stage for every dtype (64 fp16 / 128 int8 / 256 int4 elements),
//     global -> registers (16 B per lane, coalesced 128-B row segments) -> LDS, double buffered,
//     one barrier per stage; LDS rows are 128 B with a (row>>1)&7 XOR swizzle of the 16-B chunk,
//     which makes both the 8-lane row writes and the 16-row ds_read_b128 / ds_read_b64 fragment
//     reads bank-conflict free;
//   * MFMA: v_mfma_i32_16x16x64_i8 for w8a8 AND w4a4 (int4 nibbles are widened in registers to
//     16*q int8 values: hi = w & 0xF0F0F0F0, lo = (w << 4) & 0xF0F0F0F0, so the int32 sum is
//     exactly 256 * sum(a*b) and one arithmetic shift restores it: bit-exact), and
//     v_mfma_f32_16x16x32_f16 for fp16.  A and B fragments use the SAME K->(lane group, element)
//     assignment, so the (unspecified) K order inside an MFMA and the pack_wxax K permutation
//     (quantize.cuh:425-475) cancel: every product a[m,k]*b[n,k] is formed exactly once;
//   * epilogue: scale in registers, fp16 tile staged through LDS, 16-B coalesced row stores.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mxmoe {

// QT_I4G: w4a4_g128_sym (A and B int4 with one fp16 scale per 128-K group)
// QT_F8: w8a8_g-1_sym_E4M3 (A and B OCP fp8 e4m3, per-channel fp16 scales, f32 accumulate)
// QT_BF16: bf16 A and B, f32 accumulate, fp16 C
// QT_I4F6: w4a4_g-1_sym with A and B given as fp6 e3m2 images of the int4 codes (gg_f6.h): the
//          block-scaled fp6 MFMA, f32 accumulate (exact: integer partial sums below 2^24)
enum QType : int32_t {
  QT_F16 = 0, QT_I8 = 1, QT_I4 = 2, QT_W4A16 = 3, QT_W8A16 = 4, QT_I4G = 5, QT_W2A16 = 6, QT_F8 = 7, QT_BF16 = 8,
  QT_I4F6 = 9,
  QT_COUNT = 10
};
// quant types whose epilogue applies the per-channel scales sa[m] * sb[n]
constexpr bool qt_scaled(int qt) { return qt == QT_I8 || qt == QT_I4 || qt == QT_F8 || qt == QT_I4F6; }

// One row of the plan table (64 B), written by the host planner into the workspace.
struct GGMeta {
  int32_t M, N, K, qtype;
  int32_t tiles_n;     // cdiv(N, BN of this qtype)
  int32_t tile_begin;  // first global tile id of this problem
  int32_t kbytes;      // bytes of one K row (K * bits / 8; weight-only: of the fp16 A row)
  int32_t reserved;    // weight-only: 64-K stages per scale group
  int64_t lda_b, ldb_b;  // row strides of A / B in bytes
  int64_t ldc;           // row stride of C in fp16 elements
  int64_t reserved2;     // weight-only: 1 = sym codes; fp16 / w8a8 / w4a4: META_SILU
};
// GGMeta::reserved2 bit of a problem whose epilogue writes act = silu(gate) * up (MXMOE_GG_EPI_SILU_MUL):
// B rows interleaved in 16-row blocks (gate block b at rows 32 b, up block b at 32 b + 16), C has
// N / 2 columns
constexpr int64_t META_SILU = 2;
static_assert(sizeof(GGMeta) == 64, "GGMeta must stay 64 bytes");

// One output tile (32 B), host-built in dispatch order: tile b is run by workgroup b.
struct TileDesc {
  int32_t prob;  // row of the plan table; -1 = empty slot (padding of the XCD interleave)
  int32_t m0;    // first output row
  int32_t n0;    // first output column
  int32_t cls;   // bits 0-7 tile-height class; split-K: bits 8-15 slice index, bits 16-23 slices
  int32_t ks0, ks1;  // K stages [ks0, ks1) of this tile (all of K unless split)
  int32_t slab;      // split-K: first partial slab of the tile's slices, else -1
  int32_t grp;       // split-K: arrival counter of the tile, else -1
};
static_assert(sizeof(TileDesc) == 32, "TileDesc must stay 32 bytes");

// Split-K of one output tile (v2 kernels): slice `idx` of `nsplit` covers K stages
// [ks0, ks0 + nst); every slice stores its raw accumulators into its slab, the last to arrive
// sums all slabs in slice order (deterministic; int32 exact) and runs the epilogue.
constexpr int SPLITK_SLAB_BYTES = 256 * 256 * 4;  // one 256 x 256 tile of 32-bit accumulators
struct SplitK {
  int ks0, nst, idx, nsplit, slab, grp;
  uint8_t* slabs;
  int32_t* counters;
};

struct GGArgs {
  const GGMeta* meta;
  const TileDesc* tiles;
  const void* const* ptr_A;
  const void* const* ptr_B;
  const void* const* ptr_SA;
  const void* const* ptr_SB;
  void* const* ptr_C;
  int32_t P;
  int32_t n_slots;  // gridDim.x
  uint8_t* slabs;     // split-K partial slabs (SPLITK_SLAB_BYTES each)
  int32_t* counters;  // split-K arrival counters (zero between launches)
};

typedef int32_t v2i __attribute__((ext_vector_type(2)));
typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef int32_t v8i __attribute__((ext_vector_type(8)));

// Compile-time tile geometry. All dtypes stage 128 bytes of K per stage.
template <int BM_, int BN_, int WM_, int WN_, int MIN_WAVES_PER_EU_>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int kThreads = WM * WN * 64;
  static constexpr int kMinWavesPerEU = MIN_WAVES_PER_EU_;
  static constexpr int BKB = 128;  // bytes of K per stage
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int A_BYTES = BM * BKB, B_BYTES = BN * BKB;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int C_STRIDE = BN + 8;  // fp16 elements per staged C row (pad: spreads banks)
  static constexpr int C_BYTES = BM * C_STRIDE * 2;
  static constexpr int LDS_BYTES = (2 * STAGE_BYTES > C_BYTES) ? 2 * STAGE_BYTES : C_BYTES;
  static constexpr int LA = BM * 8 / kThreads;  // 16-B chunks per thread per stage (A)
  static constexpr int LB = BN * 8 / kThreads;  // (B)
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile must be a multiple of 16");
  static_assert((BM * 8) % kThreads == 0 && (BN * 8) % kThreads == 0, "stage chunks must divide threads");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// 16-B chunk `chunk` (0..7) of LDS row `row` (128-B rows), XOR-swizzled.
__device__ __forceinline__ uint32_t lds_off(int row, int chunk) {
  return (uint32_t)(row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}

// Bijective XCD-aware remap: blocks b and b+8 share an XCD under round-robin dispatch, so give
// each group of blocks {x, x+8, x+16, ...} a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7;
  const int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + (b >> 3);
}

// Widen 8 packed int4 (two's complement nibbles) per dword to int8 lanes holding 16*q.
__device__ __forceinline__ v4i widen_i4(v2i w) {
  const int32_t m = (int32_t)0xF0F0F0F0u;
  v4i r;
  r.x = w.x & m;
  r.y = (w.x << 4) & m;
  r.z = w.y & m;
  r.w = (w.y << 4) & m;
  return r;
}

template <int QT>
struct AccT {
  typedef v4i type;
};
template <>
struct AccT<QT_F16> {
  typedef v4f type;
};
template <>
struct AccT<QT_F8> {
  typedef v4f type;
};
template <>
struct AccT<QT_BF16> {
  typedef v4f type;
};
template <>
struct AccT<QT_I4F6> {
  typedef v4f type;
};

// fp8 e4m3 x e4m3 over K = 128 (one 128-B v2 stage), f32 accumulate: the block-scaled MFMA with
// every 32-element block scale = 2^0 (e8m0 code 127), i.e. the plain fp8 dot product at twice the
// bf16 MFMA rate (MI355X_MICROARCH.md, Matrix cores). Format code 0 = fp8 e4m3 for both operands.
__device__ __forceinline__ v4f mfma_f8_k128(const v8i& b, const v8i& a, const v4f& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, 0, 0, 0, 127, 0, 127);
}
__device__ __forceinline__ v8i cat_v4i(const v4i& lo, const v4i& hi) {
  return v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// One output tile of one problem.
template <class Cfg, int QT>
__device__ __forceinline__ void gg_tile(const GGMeta& mt, const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                        const _Float16* __restrict__ SA, const _Float16* __restrict__ SB,
                                        _Float16* __restrict__ C, int m0, int n0, uint8_t* lds) {
  constexpr int BM = Cfg::BM, BN = Cfg::BN, NT = Cfg::kThreads;
  constexpr int FM = Cfg::FM, FN = Cfg::FN, LA = Cfg::LA, LB = Cfg::LB;
  typedef typename AccT<QT>::type acc_t;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int rows_a = min(BM, mt.M - m0);
  const int rows_b = min(BN, mt.N - n0);
  const int kbytes = mt.kbytes;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const uint8_t* Ablk = A + (int64_t)m0 * lda;
  const uint8_t* Bblk = B + (int64_t)n0 * ldb;
  const int nstage = (kbytes + Cfg::BKB - 1) / Cfg::BKB;

  uint4 ra[LA], rb[LB];
  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  auto gload = [&](int s) {
    const int kb = s * Cfg::BKB;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + i * NT, row = q >> 3, c = q & 7;
      const bool p = (row < rows_a) && (kb + c * 16 < kbytes);
      ra[i] = p ? *reinterpret_cast<const uint4*>(Ablk + (int64_t)row * lda + kb + c * 16) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + i * NT, row = q >> 3, c = q & 7;
      const bool p = (row < rows_b) && (kb + c * 16 < kbytes);
      rb[i] = p ? *reinterpret_cast<const uint4*>(Bblk + (int64_t)row * ldb + kb + c * 16) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    uint8_t* As = lds + buf * Cfg::STAGE_BYTES;
    uint8_t* Bs = As + Cfg::A_BYTES;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int q = tid + i * NT;
      *reinterpret_cast<uint4*>(As + lds_off(q >> 3, q & 7)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int q = tid + i * NT;
      *reinterpret_cast<uint4*>(Bs + lds_off(q >> 3, q & 7)) = rb[i];
    }
  };
  auto compute = [&](int buf) {
    const uint8_t* As = lds + buf * Cfg::STAGE_BYTES;
    const uint8_t* Bs = As + Cfg::A_BYTES;
    const int r16 = lane & 15, g = lane >> 4;
    if constexpr (QT == QT_I4) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {  // 4 x 32 bytes (= 64 int4) per 128-B stage
        v4i a[FM], b[FN];
        const int chunk = 2 * s + (g >> 1), half = (g & 1) * 8;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * Cfg::WTM + i * 16 + r16;
          a[i] = widen_i4(*reinterpret_cast<const v2i*>(As + lds_off(row, chunk) + half));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * Cfg::WTN + j * 16 + r16;
          b[j] = widen_i4(*reinterpret_cast<const v2i*>(Bs + lds_off(row, chunk) + half));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {  // 2 x 64 bytes per 128-B stage
        const int chunk = kc * 4 + g;
        if constexpr (QT == QT_I8) {
          v4i a[FM], b[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i)
            a[i] = *reinterpret_cast<const v4i*>(As + lds_off(wm * Cfg::WTM + i * 16 + r16, chunk));
#pragma unroll
          for (int j = 0; j < FN; ++j)
            b[j] = *reinterpret_cast<const v4i*>(Bs + lds_off(wn * Cfg::WTN + j * 16 + r16, chunk));
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], b[j], acc[i][j], 0, 0, 0);
        } else {
          v8h a[FM], b[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i)
            a[i] = *reinterpret_cast<const v8h*>(As + lds_off(wm * Cfg::WTM + i * 16 + r16, chunk));
#pragma unroll
          for (int j = 0; j < FN; ++j)
            b[j] = *reinterpret_cast<const v8h*>(Bs + lds_off(wn * Cfg::WTN + j * 16 + r16, chunk));
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  // ---- mainloop: register-staged double buffer, one barrier per stage ----
  if (nstage > 0) {
    gload(0);
    swrite(0);
    __syncthreads();
    for (int s = 0; s < nstage; ++s) {
      const bool more = (s + 1) < nstage;
      if (more) gload(s + 1);
      compute(s & 1);
      if (more) swrite((s + 1) & 1);
      __syncthreads();
    }
  }

  // ---- epilogue: scale (quant) / round, stage the fp16 tile in LDS, coalesced 16-B stores ----
  _Float16* Cs = reinterpret_cast<_Float16*>(lds);
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (QT == QT_F16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = wm * Cfg::WTM + i * 16 + 4 * g + r, lc = wn * Cfg::WTN + j * 16 + r16;
          Cs[lr * Cfg::C_STRIDE + lc] = (_Float16)acc[i][j][r];
        }
  } else {
    constexpr int SHIFT = (QT == QT_I4) ? 8 : 0;
    _Float16 sb[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int lc = wn * Cfg::WTN + j * 16 + r16;
      sb[j] = SB[n0 + min(lc, rows_b - 1)];
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wm * Cfg::WTM + i * 16 + 4 * g + r;
        const _Float16 sa = SA[m0 + min(lr, rows_a - 1)];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int lc = wn * Cfg::WTN + j * 16 + r16;
          const _Float16 s16 = sa * sb[j];  // fp16 product, RN (mm_tile.cuh:490-493)
          // the reference rounds the product to f32 and then to fp16 (double rounding); the
          // empty asm keeps hipcc from fusing mul + cvt into one v_fma_mix (single rounding)
          float prod = (float)(acc[i][j][r] >> SHIFT) * (float)s16;
          asm volatile("" : "+v"(prod));
          const float v = 0.0f + prod;
          Cs[lr * Cfg::C_STRIDE + lc] = (_Float16)v;
        }
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per C row
#pragma unroll 4
  for (int q = tid; q < BM * CPR; q += NT) {
    const int row = q / CPR, c = q % CPR;
    if (row < rows_a && c * 8 < rows_b) {
      const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * Cfg::C_STRIDE + c * 8);
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + row) * mt.ldc + n0 + c * 8) = v;
    }
  }
  __syncthreads();  // LDS is reused by the next tile of a persistent caller
}

template <class C16, class C8, class C4>
struct FusedCfg {
  static_assert(C16::kThreads == C8::kThreads && C8::kThreads == C4::kThreads,
                "fused tiles must use the same workgroup size (compose_kernel.py:69-71)");
  static constexpr int kThreads = C16::kThreads;
  static constexpr int kMinWavesPerEU = C16::kMinWavesPerEU;
  static constexpr int m1 = C16::LDS_BYTES > C8::LDS_BYTES ? C16::LDS_BYTES : C8::LDS_BYTES;
  static constexpr int LDS_BYTES = m1 > C4::LDS_BYTES ? m1 : C4::LDS_BYTES;
};

// Fused GroupGEMM: one workgroup per tile; the qtype branch is uniform per workgroup.
template <class C16, class C8, class C4>
__global__ __launch_bounds__(C16::kThreads, C16::kMinWavesPerEU) void gg_fused_kernel(GGArgs args) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[FusedCfg<C16, C8, C4>::LDS_BYTES];
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const int lo = td.prob;
  const GGMeta mt = args.meta[lo];
  const int m_tile = td.m0, n_tile = td.n0;
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[lo]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[lo]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[lo]);
  if (mt.qtype == QT_I8) {
    gg_tile<C8, QT_I8>(mt, A, B, static_cast<const _Float16*>(args.ptr_SA[lo]),
                       static_cast<const _Float16*>(args.ptr_SB[lo]), C, m_tile, n_tile, lds);
  } else if (mt.qtype == QT_I4) {
    gg_tile<C4, QT_I4>(mt, A, B, static_cast<const _Float16*>(args.ptr_SA[lo]),
                       static_cast<const _Float16*>(args.ptr_SB[lo]), C, m_tile, n_tile, lds);
  } else {
    gg_tile<C16, QT_F16>(mt, A, B, nullptr, nullptr, C, m_tile, n_tile, lds);
  }
}


// ============================================================================================
// v2: 512-thread workgroups (8 waves, 2M x 4N), BN = 256, tile height class BM in {256, 128}.
//   * global -> LDS by LDS-DMA (global_load_lds_dwordx4): one wave-instruction fills 8 rows x
//     128 B of the lane-linear LDS image; the (row>>1)&7 chunk swizzle is applied on the SOURCE
//     address (a lane of LDS slot p of row r loads logical chunk p ^ swz(r)), the reads apply the
//     same XOR — both sides or neither (cdna_hip_programming.md rule 21);
//   * rows past M / N are clamped to the last valid row (their outputs are never stored), so no
//     load is predicated; K must be a multiple of the 128-B stage (the planner checks);
//   * two LDS stages; stage s+1 is in flight (LDS-DMA) while stage s feeds the MFMAs;
//   * MFMA operands swapped (src0 = B fragment, src1 = A fragment): each lane then owns 4
//     consecutive output COLUMNS of one row, packed into one 8-B LDS write in the epilogue;
//   * epilogue: each wave stages its own fp16 sub-tile in LDS (XOR-swizzled 16-B chunks) and
//     stores full 128-B row segments with 16-B stores.
// ============================================================================================
template <int BM_, int BN_ = 256, int WM_ = 2, int WN_ = 4>
struct V2Cfg {
  static constexpr int BM = BM_, BN = BN_, NT = 512, BKB = 128;
  static constexpr int WM = WM_, WN = WN_;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int A_BYTES = BM * BKB, B_BYTES = BN * BKB, STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int GA = BM / 64, GB = BN / 64;  // LDS-DMA wave-instructions per wave per stage
  static constexpr int EPI_BYTES = WM * WN * WTM * WTN * 2;
  static constexpr int LDS_BYTES = 2 * STAGE_BYTES > EPI_BYTES ? 2 * STAGE_BYTES : EPI_BYTES;
  static_assert(WTN == 64, "epilogue assumes 128-B staged rows");
};

// LDS beyond the two 128-KiB-image stages: the int paths' tile scales (1 KiB) and the w4a4 g128
// group-scale slots (2 x 2 KiB after a 256-row tile's two stages)
constexpr int V2_LDS_EXTRA = 4096;

typedef __attribute__((address_space(3))) void lds_void_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

// 16 zero bytes in global memory: the LDS-DMA source of K-tail chunks (they land as zeros in LDS,
// so the MFMA loop needs no tail code and no extra registers).
__device__ __attribute__((aligned(16))) const uint32_t g_zero16[4] = {0, 0, 0, 0};

// buffer-form LDS-DMA pieces (resource in SGPRs, 32-bit lane offset, soffset)
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_dst, uint32_t vo, int so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 16, vo, so, 0, 0);
}
__device__ __forceinline__ void bdma4(__amdgpu_buffer_rsrc_t rs, uint8_t* lds_dst, uint32_t vo, int so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 4, vo, so, 0, 0);
}
__device__ __forceinline__ void glds16(const void* src, uint8_t* lds_dst) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_dst, 16, 0, 0);
}

// Scaled int epilogue for the 4 columns of one accumulator fragment row:
//   fp16_rn(0 + f32(acc >> SHIFT) * f32(fp16_rn(sa * sb[c])))   (the reference's arithmetic, gg_tile)
// v_pk_mul_f16 forms two scale products at once (sa broadcast by op_sel_hi); v_fma_mix_f32 takes
// the f16 product from either half of that register and computes f32(acc) * s + 0 with ONE
// rounding, i.e. exactly the rounded f32 product, -0 turned into +0 as by the explicit add;
// v_cvt_pk_f16_f32 rounds two results to fp16. 2.75 VALU per output instead of ~5.5.
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float mul_f32_f16lo(float a, uint32_t s) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(s));
  return d;
}
__device__ __forceinline__ float mul_f32_f16hi(float a, uint32_t s) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(s));
  return d;
}
template <int SHIFT>
__device__ __forceinline__ uint2 scale_pack4(const v4i& acc, _Float16 sa, uint2 sbw) {
  const h2_t sa2 = {sa, sa};
  const uint32_t s01 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw.x));
  const uint32_t s23 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw.y));
  const h2_t lo = {(_Float16)mul_f32_f16lo((float)(acc[0] >> SHIFT), s01),
                   (_Float16)mul_f32_f16hi((float)(acc[1] >> SHIFT), s01)};
  const h2_t hi = {(_Float16)mul_f32_f16lo((float)(acc[2] >> SHIFT), s23),
                   (_Float16)mul_f32_f16hi((float)(acc[3] >> SHIFT), s23)};
  return uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}
// fp8 path: the accumulator is already f32 (no integer conversion); same scale arithmetic
__device__ __forceinline__ uint2 scale_pack4f(const v4f& acc, _Float16 sa, uint2 sbw) {
  const h2_t sa2 = {sa, sa};
  const uint32_t s01 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw.x));
  const uint32_t s23 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw.y));
  const h2_t lo = {(_Float16)mul_f32_f16lo(acc[0], s01), (_Float16)mul_f32_f16hi(acc[1], s01)};
  const h2_t hi = {(_Float16)mul_f32_f16lo(acc[2], s23), (_Float16)mul_f32_f16hi(acc[3], s23)};
  return uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}
// act = fp16(silu(f32 g) * f32 u) of 4 fp16 gate / up values, silu(g) = g * rcp(1 + exp2(-g log2 e))
// with the hardware exp2 / reciprocal: the arithmetic of the MoE activation kernel
// (moe_ops.hip act_quant_kernel, SiLU mode), so the fused epilogue's act is bit-identical to it
// (pairs in float2 vectors: the multiplies and the add issue as v_pk_mul_f32 / v_pk_add_f32 — the
// same IEEE operations, so the same bits, at half the VALU of the scalar form)
__device__ __forceinline__ uint32_t silu_mul2(uint32_t g, uint32_t u) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t gf = __builtin_convertvector(__builtin_bit_cast(h2_t, g), f2_t);
  const f2_t uf = __builtin_convertvector(__builtin_bit_cast(h2_t, u), f2_t);
  const f2_t t = gf * f2_t{-1.4426950408889634f, -1.4426950408889634f};
  const f2_t d = f2_t{1.0f, 1.0f} + f2_t{__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
  const f2_t sg = gf * f2_t{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(sg * uf, h2_t));
}
__device__ __forceinline__ uint2 silu_mul4(uint2 g, uint2 u) { return uint2{silu_mul2(g.x, u.x), silu_mul2(g.y, u.y)}; }
__device__ __forceinline__ uint2 pack4_f16(const v4f& acc) {
  const h2_t lo = {(_Float16)acc[0], (_Float16)acc[1]}, hi = {(_Float16)acc[2], (_Float16)acc[3]};
  return uint2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
}

// v_permlane16_swap: lanes 16-31 / 48-63 of x <-> lanes 0-15 / 32-47 of y (rows of 16 lanes)
__device__ __forceinline__ void swap16(uint32_t& x, uint32_t& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS barrier that lets LDS-DMA stay in flight: drain this wave's LDS reads, barrier, and keep the
// compiler from moving LDS accesses across it (the "memory" clobbers) — unlike __syncthreads(),
// no vmcnt(0).
// One 16-B row chunk of C at `base` + `off` elements, `base` wave-uniform (the wave's first output
// row / column). C is written once and never read back by the kernel, so the store carries sc1,
// which drops the line from the XCD's L2 (plain stores keep it, MI355X_MICROARCH.md "stores of each
// flavour") and leaves L2 to the A / B panels: a buffer store, base in SGPRs, 32-bit byte offset per
// lane — `narrow` (wave-uniform) says every offset of the wave fits, else a plain 64-bit store.
// Measured (profiles/r02/region/sc1_*): counter bytes -8 % on the w8a8 step, -1.4 % fp16, time
// unchanged. -DMXMOE_STORE_PLAIN builds the plain stores for A/B.
template <int AUX = 16>
__device__ __forceinline__ void store_c16(_Float16* base, int64_t off, bool narrow, const uint4& v) {
  if (narrow) {
    typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
    const v4u_ d = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(d, __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000),
                                           (int)(off * 2), 0, AUX /* 16: sc1 */);
    return;
  }
  *reinterpret_cast<uint4*>(base + off) = v;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Split-K hand-off (cdna_hip_programming.md §6 Guideline 16, counter form, write-through variant):
// every slice stores its accumulators with sc1 buffer stores (thread-linear 16-B words: coalesced;
// sc1 writes through the XCD's L2, so no agent-scope release — whose buffer_wbl2 wrote back every
// dirty line of the XCD's L2, C tiles of other blocks included — is needed), drains, and one lane
// takes the relaxed agent-scope ticket; the slice that draws nsplit - 1 re-zeroes the counter for
// the next launch and sums every slab in slice order with sc1 loads (no acquire: its buffer_inv
// emptied the XCD's L2 under the co-resident tiles' A / B panels). Returns true when `acc` holds
// the complete K sum (not split, or the last slice).
// Invariant: the slab stores and the reducing loads both carry SPLITK_AUX (sc1). The slices of one
// group may run on different XCDs (the planner's 16-entry tail chunks cut 5- and 8-slice groups;
// tests/test_planner.py::test_tail_chunks_scatter_split_slices_across_xcds pins such plans and
// tests/test_gg_gpu.py::test_splitk_slices_on_different_xcds runs them): a plain store would leave
// the partials dirty in the writer's L2, a plain load could hit a stale line in the reader's.
constexpr int SPLITK_AUX = 16;  // sc1 on both sides of the hand-off; never change one alone
template <int NT, class Acc, int FM, int FN>
__device__ __forceinline__ bool splitk_reduce(Acc (&acc)[FM][FN], const SplitK& sk, uint8_t* lds,
                                              int tid = threadIdx.x) {
  if (sk.nsplit <= 1) return true;
  static_assert(FM * FN * NT * 16 <= SPLITK_SLAB_BYTES, "tile accumulators exceed one slab");
  static_assert(sizeof(Acc) == 16, "16-B accumulator words");
  typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t mine = __builtin_amdgcn_make_buffer_rsrc(
      sk.slabs + (size_t)(sk.slab + sk.idx) * SPLITK_SLAB_BYTES, (short)0, SPLITK_SLAB_BYTES, 0x00020000);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u_, acc[i][j]), mine, ((i * FN + j) * NT + tid) * 16, 0,
                                             SPLITK_AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int32_t* flag = reinterpret_cast<int32_t*>(lds);  // the ring is drained: LDS is free here
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(sk.counters + sk.grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == sk.nsplit - 1;
    if (last) __hip_atomic_store(sk.counters + sk.grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const int last = *flag;
  __syncthreads();  // every wave has the flag before the epilogue reuses the LDS
  if (!last) return false;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = Acc{0, 0, 0, 0};
  for (int k = 0; k < sk.nsplit; ++k) {
    const __amdgpu_buffer_rsrc_t part = __builtin_amdgcn_make_buffer_rsrc(
        sk.slabs + (size_t)(sk.slab + k) * SPLITK_SLAB_BYTES, (short)0, SPLITK_SLAB_BYTES, 0x00020000);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] += __builtin_bit_cast(
            Acc, __builtin_amdgcn_raw_buffer_load_b128(part, ((i * FN + j) * NT + tid) * 16, 0, SPLITK_AUX));
  }
  return true;
}

// ABL flags. Timing ablations (results are garbage): 1 = no mainloop DMA (stage 0 reused),
// 2 = no LDS fragment reads (register fragments), 4 = no epilogue stores, 16 = every stage's
// LDS-DMA re-reads the tile's first K slice (same LDS traffic, L2-hot sources), 512 / 1024 / 2048
// (below). Options (correct results): 8 = stagger — waves 4-7 run half a stage behind waves 0-3;
// 4096 = B ring of three stages (with the stagger); 64 = tile timeline trace (diagnostics).
enum : int {
  ABL_NO_DMA = 1, ABL_NO_LDS = 2, ABL_NO_EPI = 4, V2_STAGGER = 8, ABL_DMA_HOT = 16, V2_TRACE = 64,
  ABL_B_NODMA = 512,    // ablation: B operand never loaded (A only)
  ABL_B_REGLOAD = 1024,  // ablation: B operand loaded into registers (same global traffic), not into LDS
  ABL_B_TILED = 2048,    // ablation: B read as if stored in contiguous 32-KiB (256 rows x 128 B) stage blocks
  V2_B3 = 4096,          // stagger: B in a 3-stage LDS ring, two stages ahead (A: 2 stages, one ahead)
  // spread (bits 18-20 = k): the stage's LDS-DMA pieces are issued one per k MFMAs inside the first
  // MFMA half of the stagger loop (sched_group_barrier) instead of as a burst at its top
  V2_SPREAD_SHIFT = 18,
  // buffer-form LDS-DMA: `buffer_load_dwordx4 ... lds` from a per-tile buffer resource (A / B base
  // row m0 / n0 in SGPRs), a 32-bit lane offset fixed for the whole tile and the stage's K offset in
  // soffset: no per-piece address VALU, 1 VGPR per piece instead of 2; K-tail chunks are offset
  // past num_records (the hardware returns zeros). Rows of a tile must span < 2 GiB (the planner
  // checks the row strides).
  V2_BUF = 1 << 21,
  V2_STAMP = 1 << 22,  // diagnostics (lab only): s_memtime stamps around the spread loop's waits
  // timing ablation (WRONG RESULTS by design; w4a4 tiles, staggered loop): each int4 half stage runs
  // ONE v_mfma_scale_f32_16x16x128_f8f6f4 in FP6 (e2m3) format on the raw nibble words instead of two
  // int8 MFMAs on widened nibbles: the upper bound of a w4a4 path on the FP6 MFMA (2x the int8 rate)
  ABL_I4_FP6 = 1 << 23,
  // spread option: the A pieces go one per NH/GA MFMAs of the first MFMA group, the B pieces one per
  // NH/GB MFMAs of the second (v2s3: B(s+2) has a whole stage more to land)
  V2_SPLITAB = 1 << 24,
  // spread + buffer-form option: waves 0-3 issue every LDS-DMA piece of the workgroup (their own and
  // their SIMD partner w+4's), waves 4-7 none — the stamps show the late waves are the stage's
  // critical path while the early ones wait ~1000 cycles at the barrier. Rows past M / N are read
  // out of the buffer's range (zeros) instead of clamped.
  V2_EARLYDMA = 1 << 25,
  // spread option: static priority 1 for the late waves (4-7) through the mainloop — the stamps put
  // them on the stage's critical path, the early waves wait ~1000 cycles at every barrier
  V2_PRIO_LATE = 1 << 26,
  // weight-only timing ablations (w4a16 tiles only; WRONG RESULTS by design): B read from 8-KiB
  // stage blocks / no LDS-DMA after the ring's first fill / no fragment reads, dequant or MFMA
  ABL_WO_BTILED = 1 << 14, ABL_WO_NODMA = 2 << 14, ABL_WO_NOCOMPUTE = 4 << 14,
  // weight-only option (correct results): the 128 / 64-row tiles read stage s+1's fragments into a
  // second register set right after the barrier that publishes it, and run stage s's dequant +
  // MFMAs while those reads are in flight (gg_tile_wo)
  WO_PIPE = 1 << 17,
  // with WO_PIPE: waves 4-7 defer each stage's second-K-half MFMAs (operands dequantised before
  // the barrier, held in registers) past the next barrier, so SIMD partners are half a stage
  // apart — one wave's MFMAs beside the other's dequant VALU. Accumulation order unchanged.
  WO_STAG = 1 << 27,
  // epilogue option: each wave writes fragment row i of its sub-tile into its LDS region, then
  // reads back and stores fragment row i - 1 (16 rows), so the C stores start after one eighth of
  // the scale / pack VALU instead of after all of it and drain under the rest
  V2_EPIPE = 1 << 28,
  // spread + EDMA option: the late waves interleave the A-fragment reads of the next K half into the
  // current MFMA group (one read after the 4 MFMAs of each fragment row, which frees that row's
  // registers), leaving only the B reads between the last MFMA and the barrier
  V2_LATEIL = 1 << 29,
  // epilogue option: plain C stores instead of sc1 (tools/store_probe.hip: a 128-KiB tile drains in
  // 1366 vs 2434 cycles with 32 CUs storing). MEASURED NEGATIVE (round 4): C straight from the
  // accumulator registers (pairs of 16 x 16 blocks exchanged by v_permlane16_swap, 16 rows x 64 B per
  // store instruction): 13-15 % slower than the LDS-staged 8 rows x 128 B (probe: 5219 vs 2434 cycles
  // per tile), profiles/r04/lab_a/
  V2_PLAINST = 1 << 30,
  // int4 option (lab): an empty asm statement between the staggered loop's 8-B fragment reads, so
  // hipcc cannot pair them into ds_read2st64_b64 (2-way bank conflicts on every pair; the bit is
  // WO_SCLATE's, a gg_tile_wo option the v2 int4 body never sees)
  V2_I4NOPAIR = 32,
  // weight-only option (non-pipelined loop, wo3): a stage that opens a scale group brings the
  // group's scale words by LDS-DMA into a slot beside its ring buffer, covered by the stage's own
  // counted wait (round 3 loaded them into registers right before use: the compiler's vmcnt(0)
  // drained the whole ring at every group boundary, every second stage at g128); group positions
  // and ring indices are counters, not a division / modulo per stage
  WO_SCLATE = 32,
  // weight-only option: the code -> fp16 constants in registers (WoK): one v_and_or_b32 per fp16
  // pair (4 / 2-bit codes), one v_perm_b32 (8-bit) — VALU-bound small-batch tiles
  WO_ANDOR = 128,
  // with V2_TRACE (lab diagnostics, v2 staggered + B3 loop): the trace's second mark is taken after
  // the prologue barrier (stage 0 landed) instead of after the mainloop, so the tile timeline splits
  // off the prologue (the bit is WO_ANDOR's, which gg_v2_kernel never passes to a v2 body)
  V2_TRACE_PRO = 128,
  // with V2_TRACE (lab diagnostics): the second mark is taken once the tile's descriptor, problem
  // metadata and operand pointers are in registers, right before the prologue's first LDS-DMA
  // (the bit is WO_MSKIP's, which gg_v2_kernel never passes to a v2 body)
  V2_TRACE_DESC = 256,
  // lab option: the early-wave DMA issue (V2_EARLYDMA) on int4 tiles too (round 3 measured it 2.5-4.3 %
  // slower on w4a4, before the int4 reads were unpaired; the bit is WO_SPLIT's, which gg_v2_kernel
  // never passes to a v2 body)
  V2_I4EDMA = 8192,
  // weight-only option (non-pipelined loop): skip the MFMAs and A reads of 16-row blocks wholly past M
  WO_MSKIP = 256,
  // with WO_SCLATE: the steady state (stage s + DIST exists) and the tail as two loops
  WO_SPLIT = 8192,
  // weight-only option: 4 / 2-bit codes converted where they sit (WoK::nibpos)
  WO_NIBPOS = INT32_MIN,
  // with WO_SCLATE | WO_SPLIT: waves whose A rows all lie past M issue no A piece (gg_tile_wo;
  // the bit is ABL_B_TILED's, an int8-only v2 ablation gg_tile_wo never sees). MEASURED NEGATIVE
  // (round 4, lab): 0.5-2.5 % slower on the bs 512 calls (profiles/r04/wo/wo_i)
  WO_ADEAD = 2048,
  // weight-only option: buffer-form LDS-DMA in gg_tile_wo (the bit is ABL_DMA_HOT's, a v2-only
  // ablation gg_tile_wo never sees)
  WO_BUF = 16
};
constexpr int kWoAblMask = ABL_WO_BTILED | ABL_WO_NODMA | ABL_WO_NOCOMPUTE;
// weight-only option (round 6): the fused SiLU epilogue (MXMOE_GG_EPI_SILU_MUL, epilogue_v3's SiLU
// path) compiled into gg_tile_wo — a separate wo2 instantiation, launched only for calls whose
// weight-only problems carry the flag, so the plain 3-WG/CU build keeps its registers (the bit is
// V2_EPIPE's, a v2 epilogue option no weight-only tile sees)
constexpr int WO_SILU = 1 << 28;
// weight-only option (round 6, with WO_SCLATE | WO_SPLIT): a tile whose K stages lie in ONE scale group
// (per-channel scales — the small-batch bench scheme's w4a16_g-1) runs a loop without the group
// bookkeeping, unrolled by the ring depth so the ring offsets are constants (the bit is V2_SPREAD's
// lowest, a v2 option no weight-only tile sees)
constexpr int WO_PCH = 1 << 18;

// f(integral_constant<int, I>) for I in [I0, N)
template <int I0, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I0 < N) {
    f(std::integral_constant<int, I0>());
    static_for<I0 + 1, N>(f);
  }
}
constexpr int kAblMask = ABL_NO_DMA | ABL_NO_LDS | ABL_NO_EPI | ABL_B_NODMA | ABL_B_REGLOAD | ABL_B_TILED;  // int8-only builds

// Tile timeline (diagnostics, V2_TRACE builds only): per block {start, mainloop end, end (stores
// drained), nst << 48 | class << 40 | qtype << 36 | XCC_ID << 32 | HW_ID}, s_memrealtime ticks
// (100 MHz); read back with mxmoe_gg_debug_trace.
constexpr int kTraceBlocks = 32768;
__device__ uint64_t g_gg_trace[kTraceBlocks * 4];
#ifdef MXMOE_LAB
// per-wave stage stamps of the spread mainloop (V2_STAMP builds, lab library only): per (block, wave)
// {sum of s_memtime cycles in the stage body, in the vmcnt(0) wait, in the barrier, steady stages}
constexpr int kStampBlocks = 4096;
__device__ uint64_t g_gg_stamp[kStampBlocks * 8 * 4];
#endif
__device__ __forceinline__ void trace_mark(int slot) {
  if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks) g_gg_trace[blockIdx.x * 4 + slot] = __builtin_amdgcn_s_memrealtime();
}

// One 64-B K half of a v2 stage (128-B rows, XOR-swizzled 16-B chunks) as raw fragment words:
// read from LDS, then consumed by the MFMAs (int4 widened at use). Used by the staggered v2
// mainloop (gg_tile_v2 with V2_STAGGER).
// One operand's 128-B K stage of G x 8 rows per wave into a lane-linear LDS image (v2 layout); the
// K tail (last stage only) loads 16 zero bytes for chunks past K.
template <int G>
__device__ __forceinline__ void v2_dma(const uint8_t* const (&src)[G], uint8_t* dst, int kb, int kbytes, int wave,
                                       int lane) {
  if (kb + 128 <= kbytes) {
#pragma unroll
    for (int j = 0; j < G; ++j) glds16(src[j] + kb, dst + (wave * G + j) * 1024);
  } else {
    const int rsub = lane >> 3, p = lane & 7;
    const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero16);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int kc = (p ^ ((((wave * G + j) * 8 + rsub) >> 1) & 7)) << 4;
      glds16(kb + kc < kbytes ? src[j] + kb : zero, dst + (wave * G + j) * 1024);
    }
  }
}

template <class Cfg, int QT, int ABL = 0>
struct V2Half {
  // int4: 8-B reads per MFMA K step (hipcc pairs them into ds_read2st64_b64, 2-way bank conflicts:
  // the 16-B form of gg_tile_v3 / the plain v2 loop adds the registers of the second step's words to
  // the staggered loop, which sits at 254 VGPRs, and spilled there — DESIGN.md §7 round 5)
  typedef typename std::conditional<QT == QT_I4, v2i, v4i>::type word_t;
  static constexpr int FM = Cfg::FM, FN = Cfg::FN;
  static constexpr int SUBH = (QT == QT_I4) ? 2 : 1;  // MFMA K steps per 64-B half stage
  static constexpr int kMfma = SUBH * FM * FN, kReads = SUBH * (FM + FN);  // per half stage
  word_t a[SUBH][FM];
  word_t b[SUBH][FN];

  __device__ __forceinline__ void read(const uint8_t* abase, const uint8_t* bbase, uint32_t a_row, uint32_t b_row, int swz,
                                       int g, int h) {
    const uint8_t* As = abase + a_row;
    const uint8_t* Bs = bbase + b_row;
#pragma unroll
    for (int t = 0; t < SUBH; ++t) {
      const uint32_t off = QT == QT_I4 ? (uint32_t)(((2 * (2 * h + t) + (g >> 1)) ^ swz) << 4) + (uint32_t)((g & 1) * 8)
                                       : (uint32_t)(((h * 4 + g) ^ swz) << 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        a[t][i] = *reinterpret_cast<const word_t*>(As + i * 2048 + off);
        if constexpr (QT == QT_I4 && (ABL & V2_I4NOPAIR) != 0) asm volatile("");
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        b[t][j] = *reinterpret_cast<const word_t*>(Bs + j * 2048 + off);
        if constexpr (QT == QT_I4 && (ABL & V2_I4NOPAIR) != 0) asm volatile("");
      }
    }
  }
  __device__ __forceinline__ void mma(typename AccT<QT>::type (&acc)[FM][FN]) const {
    if constexpr (QT == QT_I4 && (ABL & ABL_I4_FP6) != 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const v8i aw = {a[0][i][0], a[0][i][1], a[1][i][0], a[1][i][1], a[0][i][0] ^ a[1][i][1], a[0][i][1], 0, 0};
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const v8i bw = {b[0][j][0], b[0][j][1], b[1][j][0], b[1][j][1], b[0][j][0] ^ b[1][j][1], b[0][j][1], 0, 0};
          acc[i][j] = __builtin_bit_cast(
              v4i, __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bw, aw, __builtin_bit_cast(v4f, acc[i][j]), 2, 2, 0,
                                                                    127, 0, 127));
        }
      }
      return;
    }
#pragma unroll
    for (int t = 0; t < SUBH; ++t) {
      if constexpr (QT == QT_I4) {
        v4i bw[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) bw[j] = widen_i4(b[t][j]);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const v4i aw = widen_i4(a[t][i]);
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bw[j], aw, acc[i][j], 0, 0, 0);
        }
      } else if constexpr (QT == QT_I8) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[t][j], a[t][i], acc[i][j], 0, 0, 0);
      } else if constexpr (QT == QT_BF16) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, b[t][j]),
                                                                __builtin_bit_cast(v8bf, a[t][i]), acc[i][j], 0, 0, 0);
      } else {
        static_assert(QT == QT_F16, "V2Half: fp8 tiles run the plain v2 mainloop (one K=128 MFMA per stage)");
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, b[t][j]),
                                                               __builtin_bit_cast(v8h, a[t][i]), acc[i][j], 0, 0, 0);
      }
    }
  }
};

template <class Cfg, int QT, int ABL = 0>
__device__ __forceinline__ void gg_tile_v2(const GGMeta& mt, const uint8_t* __restrict__ A,
                                           const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                           const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0, int n0,
                                           uint8_t* lds, const SplitK& sk) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB;
  typedef typename AccT<QT>::type acc_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N, kbytes = mt.kbytes;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = sk.nst, ks0 = sk.ks0;  // this tile's K stages [ks0, ks0 + nst) (all of K unless split)

  // per-lane LDS-DMA sources (row clamped, chunk pre-swizzled); + kb per stage
  const uint8_t* srcA[GA];
  const uint8_t* srcB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      const int grow = min(m0 + row, M - 1);
      srcA[j] = A + (int64_t)grow * lda + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      const int grow = min(n0 + row, N - 1);
      srcB[j] = B + (int64_t)grow * ldb + ((p ^ ((row >> 1) & 7)) << 4);
      if constexpr ((ABL & ABL_B_TILED) != 0)  // block (n0/256, stage) at ((n0/256)*nstages + stage)*32 KiB
        srcB[j] = B + (int64_t)(n0 / 256) * ((kbytes + 127) / 128) * 32768 + row * 128 + ((p ^ ((row >> 1) & 7)) << 4);
    }
  }
  // V2_BUF: per-tile buffer resources and fixed 32-bit lane offsets (rows relative to m0 / n0)
  // (V2_EARLYDMA: num_records ends at row M / N, rows past it read as zeros; else rows are clamped)
  constexpr bool kOobRows = (ABL & V2_EARLYDMA) != 0;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(A) + (int64_t)m0 * lda, (short)0,
      kOobRows ? (int)(min(M - m0, Cfg::BM) * lda) : 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(B) + (int64_t)n0 * ldb, (short)0,
      kOobRows ? (int)(min(N - n0, Cfg::BN) * ldb) : 0x7fffffff, 0x00020000);
  uint32_t voA[GA], voB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      voA[j] = (uint32_t)((kOobRows ? row : min(m0 + row, M - 1) - m0) * lda) + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      voB[j] = (uint32_t)((kOobRows ? row : min(n0 + row, N - 1) - n0) * ldb) + ((p ^ ((row >> 1) & 7)) << 4);
    }
  }
  auto bdma = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t vo, int kb, uint8_t* dst) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)dst, 16, vo, kb, 0, 0);
  };
  uint4 breg[GB];  // ABL_B_REGLOAD sink
  auto issue = [&](int s, int buf) {
    if constexpr ((ABL & ABL_NO_DMA) != 0) {
      if (s > 0) return;
    }
    uint8_t* As = lds + buf * Cfg::STAGE_BYTES;
    uint8_t* Bs = As + Cfg::A_BYTES;
    const int kb = (ABL & ABL_DMA_HOT) ? ks0 * Cfg::BKB : (ks0 + s) * Cfg::BKB;
    if constexpr ((ABL & V2_BUF) != 0) {
      const bool full = kb + Cfg::BKB <= kbytes;
      const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int kc = (p ^ ((((wave * GA + j) * 8 + rsub) >> 1) & 7)) << 4;
        bdma(rsA, full || kb + kc < kbytes ? voA[j] : 0x80000000u, kb, As + (wave * GA + j) * 1024);
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int kc = (p ^ ((((wave * GB + j) * 8 + rsub) >> 1) & 7)) << 4;
        bdma(rsB, full || kb + kc < kbytes ? voB[j] : 0x80000000u, kb, Bs + (wave * GB + j) * 1024);
      }
      return;
    }
    if (kb + Cfg::BKB <= kbytes) {
#pragma unroll
      for (int j = 0; j < GA; ++j) glds16(srcA[j] + kb, As + (wave * GA + j) * 1024);
      if constexpr ((ABL & ABL_B_REGLOAD) != 0) {
#pragma unroll
        for (int j = 0; j < GB; ++j) breg[j] = *reinterpret_cast<const uint4*>(srcB[j] + kb);
      } else if constexpr ((ABL & ABL_B_TILED) != 0) {
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(srcB[j] + (int64_t)kb * 256, Bs + (wave * GB + j) * 1024);
      } else if constexpr ((ABL & ABL_B_NODMA) == 0) {
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16(srcB[j] + kb, Bs + (wave * GB + j) * 1024);
      }
    } else {
      // K tail (last stage only): chunks past K load 16 zero bytes instead
      const int rsub = lane >> 3, p = lane & 7;
      const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero16);
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int kc = (p ^ ((((wave * GA + j) * 8 + rsub) >> 1) & 7)) << 4;
        glds16(kb + kc < kbytes ? srcA[j] + kb : zero, As + (wave * GA + j) * 1024);
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int kc = (p ^ ((((wave * GB + j) * 8 + rsub) >> 1) & 7)) << 4;
        glds16(kb + kc < kbytes ? srcB[j] + kb : zero, Bs + (wave * GB + j) * 1024);
      }
    }
  };

  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  const int swz = (r16 >> 1) & 7;  // rows of a fragment are base + r16 with base % 16 == 0
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u;
  const uint32_t b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  // a wave whose rows all lie past M (the small-batch 64 x 128 tiles' 16-row waves on ~35-row
  // experts) skips its fragment reads and MFMAs; its accumulators stay zero and are never stored
#ifndef MXMOE_V2_NO_WSKIP
  const bool wave_dead = m0 + wm * Cfg::WTM >= M;
#else
  const bool wave_dead = false;
#endif
  auto compute = [&](int buf) {
    if (wave_dead) return;
    const uint8_t* As = lds + buf * Cfg::STAGE_BYTES + a_row;
    const uint8_t* Bs = lds + buf * Cfg::STAGE_BYTES + Cfg::A_BYTES + b_row;
    if constexpr (QT == QT_F8) {
      // one K = 128 MFMA per fragment pair and stage: lane group g holds the 16-B chunks g and g + 4
      // (the int8 path's two K halves), the same K assignment for A and B
      const uint32_t off0 = (uint32_t)((g ^ swz) << 4), off1 = (uint32_t)(((4 + g) ^ swz) << 4);
      v8i b[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = cat_v4i(*reinterpret_cast<const v4i*>(Bs + j * 2048 + off0), *reinterpret_cast<const v4i*>(Bs + j * 2048 + off1));
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const v8i a = cat_v4i(*reinterpret_cast<const v4i*>(As + i * 2048 + off0),
                              *reinterpret_cast<const v4i*>(As + i * 2048 + off1));
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_f8_k128(b[j], a, acc[i][j]);
      }
    } else if constexpr (QT == QT_I4) {
      // two 64-B halves; lane group g reads chunk (4 kc + g) ^ swz (16 B, as the int8 path) and
      // runs two MFMA K steps on its 8-B halves (V2Half: the same K map for A and B)
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const uint32_t off = (uint32_t)(((kc * 4 + g) ^ swz) << 4);
        v4i a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v4i*>(As + i * 2048 + off);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v4i*>(Bs + j * 2048 + off);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          v4i bw[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) bw[j] = widen_i4(v2i{b[j][2 * t], b[j][2 * t + 1]});
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const v4i aw = widen_i4(v2i{a[i][2 * t], a[i][2 * t + 1]});
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bw[j], aw, acc[i][j], 0, 0, 0);
          }
        }
      }
    } else {
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) {
        const uint32_t off = (uint32_t)(((kc * 4 + g) ^ swz) << 4);
        if constexpr (QT == QT_I8) {
          v4i a[FM], b[FN];
          if constexpr ((ABL & ABL_NO_LDS) != 0) {
#pragma unroll
            for (int i = 0; i < FM; ++i) {
              a[i] = v4i{lane + i, kc, buf, 7};
              asm volatile("" : "+v"(a[i]));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              b[j] = v4i{lane - j, kc, 3, buf};
              asm volatile("" : "+v"(b[j]));
            }
          } else {
#pragma unroll
            for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v4i*>(As + i * 2048 + off);
#pragma unroll
            for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v4i*>(Bs + j * 2048 + off);
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
        } else if constexpr (QT == QT_BF16) {
          v8bf a[FM], b[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v8bf*>(As + i * 2048 + off);
#pragma unroll
          for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v8bf*>(Bs + j * 2048 + off);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        } else {
          v8h a[FM], b[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v8h*>(As + i * 2048 + off);
#pragma unroll
          for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v8h*>(Bs + j * 2048 + off);
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a[i], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  // int paths: row / column scales of the tile -> LDS (after the mainloop's LDS area). The load
  // is issued with stage 0's DMA and written after the prologue barrier, so its latency hides
  // under stage 0's and no register stays live across the mainloop.
  _Float16 sc = 0;
  if constexpr (qt_scaled(QT)) {
    if (tid < Cfg::BM) sc = SA[min(m0 + tid, M - 1)];
    else if (tid >= 256) sc = SB[min(n0 + tid - 256, N - 1)];
  }
  auto stash_scale = [&]() {
    if constexpr (qt_scaled(QT)) {
      if (tid < Cfg::BM || tid >= 256) reinterpret_cast<_Float16*>(lds + Cfg::LDS_BYTES)[tid] = sc;
    }
  };

  // ---- stagger (V2_STAGGER): SIMD partners are waves w and w+4 (a workgroup's waves go to the
  // SIMDs cyclically). In lockstep both read LDS, then both issue MFMAs, then meet at the barrier.
  // Waves 4-7 instead defer the second K half of every stage past the barrier, holding its
  // fragments in registers: after each barrier they start on MFMAs while waves 0-3 start on LDS
  // reads. Every accumulator still sees its K chunks in order -> bit-identical results.
  if constexpr ((ABL & V2_STAGGER) != 0 && ((ABL >> V2_SPREAD_SHIFT) & 7) != 0) {
    // Staggered v2 with the stage's LDS-DMA spread over the MFMAs. Each steady-state iteration (every
    // piece it issues is a full 128-B stage) is one basic block, ordered by sched_group_barrier as
    //   early waves: ds_read half 0 | {k MFMA, 1 DMA piece} x (GA+GB) | rest of half 0 | ds_read half 1 | MFMA half 1
    //   late waves:  {1 DMA piece, k MFMA} x (GA+GB) | rest of the deferred half | ds_read | MFMA | ds_read
    // then the stage-end wait + barrier. Two LDS images: v2s (both operands one stage ahead, two
    // 64-KiB stages, vmcnt(0)) or, with V2_B3, v2s3 (A one stage ahead in a 2-stage ring, B two
    // stages ahead in a 3-stage ring; the A pieces are issued first, so vmcnt(GB) leaves exactly
    // B(s+2) in flight). The K-tail stages and the late waves' first stage run the plain bodies.
    typedef V2Half<Cfg, QT, ABL> Half;
    constexpr bool B3 = (ABL & V2_B3) != 0;
    constexpr int NH = Half::kMfma, NR = Half::kReads, ND = GA + GB;
    constexpr int KS0 = (ABL >> V2_SPREAD_SHIFT) & 7, KS = KS0 * ND <= NH ? KS0 : NH / ND;  // small tiles: denser
    static_assert(KS >= 1, "spread: more DMA pieces than MFMAs in a half stage");
    constexpr int KSA = NH / GA, KSB = NH / GB;  // V2_SPLITAB: A pieces over group 1, B over group 2
    auto abuf = [&](int t) -> uint8_t* {
      return B3 ? lds + (t & 1) * Cfg::A_BYTES : lds + (t & 1) * Cfg::STAGE_BYTES;
    };
    auto bbuf = [&](int t) -> uint8_t* {
      return B3 ? lds + 2 * Cfg::A_BYTES + (t % 3) * Cfg::B_BYTES : lds + (t & 1) * Cfg::STAGE_BYTES + Cfg::A_BYTES;
    };
    // one operand's pieces of stage t; `full`: no K tail in this stage (no per-lane select)
    // (not on int4 tiles: their half stages carry twice the MFMAs, the early waves have no slack —
    //  w4a4 2.5-4.3 % slower with it, profiles/r03/lab/lab_r3.jsonl)
    constexpr bool EDMA = (ABL & V2_EARLYDMA) != 0 && (QT != QT_I4 || (ABL & V2_I4EDMA) != 0);
    static_assert(!EDMA || (ABL & V2_BUF) != 0, "V2_EARLYDMA needs the buffer-form DMA");
    constexpr int HALFW = Cfg::WM * Cfg::WN / 2;  // SIMD partner of wave w is w + HALFW
    // one operand's pieces of stage t; `full`: no K tail in this stage (no per-lane select).
    // EDMA: early waves issue their partner's pieces too (rows + 8 * G * HALFW, the same swizzle),
    // late waves none; `early` is a constant after inlining into either wave's loop.
    auto dma_a = [&](int t, bool full, bool early) {
      const int kb = (ks0 + t) * Cfg::BKB, rsub = lane >> 3, p = lane & 7;
      uint8_t* dst = abuf(t);
      if (EDMA && !early) return;
#pragma unroll
      for (int w2 = 0; w2 < (EDMA ? 2 : 1); ++w2) {
        const int ww = wave + w2 * HALFW;
        const uint32_t radd = (uint32_t)(w2 * 8 * GA * HALFW * lda);
#pragma unroll
        for (int j = 0; j < GA; ++j) {
          const int kc = (p ^ ((((wave * GA + j) * 8 + rsub) >> 1) & 7)) << 4;
          const bool in = full || kb + kc < kbytes;
          if constexpr ((ABL & V2_BUF) != 0) bdma(rsA, in ? voA[j] + radd : 0x80000000u, kb, dst + (ww * GA + j) * 1024);
          else glds16(in ? srcA[j] + kb : reinterpret_cast<const uint8_t*>(g_zero16), dst + (wave * GA + j) * 1024);
        }
      }
    };
    auto dma_b = [&](int t, bool full, bool early) {
      const int kb = (ks0 + t) * Cfg::BKB, rsub = lane >> 3, p = lane & 7;
      uint8_t* dst = bbuf(t);
      if (EDMA && !early) return;
#pragma unroll
      for (int w2 = 0; w2 < (EDMA ? 2 : 1); ++w2) {
        const int ww = wave + w2 * HALFW;
        const uint32_t radd = (uint32_t)(w2 * 8 * GB * HALFW * ldb);
#pragma unroll
        for (int j = 0; j < GB; ++j) {
          const int kc = (p ^ ((((wave * GB + j) * 8 + rsub) >> 1) & 7)) << 4;
          const bool in = full || kb + kc < kbytes;
          if constexpr ((ABL & V2_BUF) != 0) bdma(rsB, in ? voB[j] + radd : 0x80000000u, kb, dst + (ww * GB + j) * 1024);
          else glds16(in ? srcB[j] + kb : reinterpret_cast<const uint8_t*>(g_zero16), dst + (wave * GB + j) * 1024);
        }
      }
    };
    const int nst_full = (ks0 + nst) * Cfg::BKB > kbytes ? nst - 1 : nst;  // stages [0, nst_full) are full
    auto full_stage = [&](int t) { return t < nst_full; };
    // the pieces issued in iteration s (v2s: A(s+1), B(s+1); v2s3: A(s+1), B(s+2)), full stages only
    auto dma_steady = [&](int s, bool early) {
      dma_a(s + 1, true, early);
      dma_b(s + (B3 ? 2 : 1), true, early);
    };
    auto dma_generic = [&](int s, bool early) {
      if (s + 1 < nst) dma_a(s + 1, full_stage(s + 1), early);
      const int tb = s + (B3 ? 2 : 1);
      if (tb < nst) dma_b(tb, full_stage(tb), early);
    };
    // iterations s < nsteady issue only full stages
    const int nsteady = nst_full - (B3 ? 2 : 1);
    auto stage_wait = [&](int s) {  // stage s+1 landed (B3: B(s+2) may stay in flight)
      if (B3 && s + 2 < nst) wait_vmcnt<(EDMA ? 2 : 1) * GB>();
      else wait_vmcnt<0>();
    };
    // EDMA: the early waves carry twice the pieces, the late ones none
    // (64-row tiles: more pieces than MFMAs in a half stage -> one MFMA per piece, the rest of the
    // pieces run into the second group)
    constexpr int NDE = EDMA ? 2 * ND : ND;
    constexpr int KSE = KS0 * NDE <= NH ? KS0 : (NH / NDE > 0 ? NH / NDE : 1);
    constexpr int RESTE = NH - KSE * NDE > 0 ? NH - KSE * NDE : 0;
    auto hread = [&](Half& f, int t, int h) { f.read(abuf(t), bbuf(t), a_row, b_row, swz, g, h); };
    auto hmma = [&](const Half& f) { f.mma(acc); };
    // V2_STAMP: body = loop top -> every MFMA issued (sched_barrier), vm = the stage-end vmcnt wait,
    // bar = the barrier
    [[maybe_unused]] auto stamped_sync = [&](int s, uint64_t t0, uint64_t& body, uint64_t& vm, uint64_t& bar) {
      __builtin_amdgcn_sched_barrier(0);
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      stage_wait(s);
      const uint64_t t2 = __builtin_amdgcn_s_memtime();
      lds_barrier();
      const uint64_t t3 = __builtin_amdgcn_s_memtime();
      body += t1 - t0;
      vm += t2 - t1;
      bar += t3 - t2;
    };
    [[maybe_unused]] auto stamp_out = [&](uint64_t body, uint64_t vm, uint64_t bar, int n) {
#ifdef MXMOE_LAB
      if (lane == 0 && blockIdx.x < kStampBlocks && n > 0) {
        uint64_t* o = g_gg_stamp + ((size_t)blockIdx.x * 8 + wave) * 4;
        o[0] = body;
        o[1] = vm;
        o[2] = bar;
        o[3] = (uint64_t)n;
      }
#endif
    };
    // the last stage's second 64-B half lies wholly past K (e.g. int4 at K = 1408: 704 B, 5.5 stages):
    // its fragments are the DMA's zero fill, so neither wave group reads them or runs their MFMAs
    // (products with zeros: the int32 sums are unchanged; f32 ones at most the sign of an exact zero)
    const bool last_h1_empty = nst > 0 && (ks0 + nst - 1) * Cfg::BKB + Cfg::BKB / 2 >= kbytes;
    if (nst > 0) {
      Half fr;
      // prologue: stage 0 (and B3: B(1)) in flight, then the first barrier
      const bool early_w = wave < HALFW;
      if constexpr ((ABL & V2_TRACE) != 0 && (ABL & V2_TRACE_DESC) != 0) {
        asm volatile("" ::"s"(A), "s"(B), "s"(lda), "s"(ldb), "s"(kbytes), "s"(M), "s"(N));
        trace_mark(1);
      }
      dma_a(0, full_stage(0), early_w);
      dma_b(0, full_stage(0), early_w);
      if (B3 && nst > 1) dma_b(1, full_stage(1), early_w);
      stage_wait(-1);
      lds_barrier();
      if constexpr ((ABL & V2_TRACE) != 0 && (ABL & V2_TRACE_PRO) != 0) trace_mark(1);
      if constexpr (!B3) stash_scale();  // (B3: the rings fill the LDS, the stash follows the mainloop)
      uint64_t st_body = 0, st_vm = 0, st_bar = 0;
#ifndef MXMOE_V2_NO_LATEDEAD
      // every row of the late waves lies past M (a tail tile of <= BM / 2 rows: the int paths'
      // 128-row class holding <= 64): with EDMA they issue no DMA piece either, so they skip their
      // fragment reads and MFMAs and only keep the barrier count (one per stage, as below)
      const bool late_dead = EDMA && Cfg::WM % 2 == 0 && M - m0 <= Cfg::BM / 2;
#else
      const bool late_dead = false;
#endif
      if (wave >= Cfg::WM * Cfg::WN / 2 && late_dead) {
        for (int s = 0; s < nst; ++s) lds_barrier();
      } else if (wave >= Cfg::WM * Cfg::WN / 2) {  // late waves
        if constexpr ((ABL & V2_PRIO_LATE) != 0) __builtin_amdgcn_s_setprio(1);
        dma_generic(0, false);
        hread(fr, 0, 0);
        hmma(fr);
        hread(fr, 0, 1);
        stage_wait(0);
        lds_barrier();
        int s = 1;
        for (; s < nsteady; ++s) {
          [[maybe_unused]] uint64_t t0 = 0;
          if constexpr ((ABL & V2_STAMP) != 0) t0 = __builtin_amdgcn_s_memtime();
          dma_steady(s, false);
          hmma(fr);  // second half of stage s-1
          hread(fr, s, 0);
          hmma(fr);
          hread(fr, s, 1);
          if constexpr (EDMA && (ABL & V2_LATEIL) != 0 && Half::SUBH == 1) {
            // {FN MFMAs of fragment row i, the next half's read of a[i]} x FM, then the FN B reads
#pragma unroll
            for (int q = 0; q < 2; ++q) {
#pragma unroll
              for (int i = 0; i < FM; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              }
              __builtin_amdgcn_sched_group_barrier(0x100, FN, 0);
            }
          } else if constexpr (EDMA) {
            __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          } else if constexpr ((ABL & V2_SPLITAB) != 0) {
#pragma unroll
            for (int q = 0; q < GA; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, KSA, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KSA * GA, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
            for (int q = 0; q < GB; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, KSB, 0);
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KSB * GB, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          } else {
#pragma unroll
            for (int q = 0; q < ND; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KS * ND, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          }
          if constexpr ((ABL & V2_STAMP) != 0) {
            stamped_sync(s, t0, st_body, st_vm, st_bar);
          } else {
            stage_wait(s);
            lds_barrier();
          }
        }
        if constexpr ((ABL & V2_STAMP) != 0) stamp_out(st_body, st_vm, st_bar, nsteady - 1);
        for (; s < nst; ++s) {
          dma_generic(s, false);
          hmma(fr);
          hread(fr, s, 0);
          hmma(fr);
          hread(fr, s, 1);
          stage_wait(s);
          lds_barrier();
        }
        if (!last_h1_empty) hmma(fr);  // the deferred second half of the last stage (zeros: skipped)
        if constexpr ((ABL & V2_PRIO_LATE) != 0) __builtin_amdgcn_s_setprio(0);
      } else {  // early waves
        int s = 0;
        for (; s < nsteady; ++s) {
          [[maybe_unused]] uint64_t t0 = 0;
          if constexpr ((ABL & V2_STAMP) != 0) t0 = __builtin_amdgcn_s_memtime();
          hread(fr, s, 0);
          dma_steady(s, true);
          hmma(fr);
          hread(fr, s, 1);
          hmma(fr);
          __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          if constexpr (EDMA) {
#pragma unroll
            for (int q = 0; q < NDE; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, KSE, 0);
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, RESTE, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
          } else if constexpr ((ABL & V2_SPLITAB) != 0) {
#pragma unroll
            for (int q = 0; q < GA; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, KSA, 0);
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KSA * GA, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
            for (int q = 0; q < GB; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, KSB, 0);
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KSB * GB, 0);
          } else {
#pragma unroll
            for (int q = 0; q < ND; ++q) {
              __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
              __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NH - KS * ND, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
          }
          if constexpr ((ABL & V2_STAMP) != 0) {
            stamped_sync(s, t0, st_body, st_vm, st_bar);
          } else {
            stage_wait(s);
            lds_barrier();
          }
        }
        if constexpr ((ABL & V2_STAMP) != 0) stamp_out(st_body, st_vm, st_bar, nsteady);
        for (; s < nst; ++s) {
          dma_generic(s, true);
          hread(fr, s, 0);
          hmma(fr);
          if (!(last_h1_empty && s == nst - 1)) {
            hread(fr, s, 1);
            hmma(fr);
          }
          stage_wait(s);
          lds_barrier();
        }
      }
    }
    if constexpr (B3) {
      stash_scale();  // the rings are dead: the scale stash (past the epilogue image) is free
      if constexpr (qt_scaled(QT)) __syncthreads();
    }
  } else if constexpr ((ABL & V2_STAGGER) != 0 && (ABL & V2_B3) != 0) {
    // B3: A ring of 2 stages at [0, 2 A_BYTES), B ring of 3 at [2 A_BYTES, + 3 B_BYTES). Stage s+1's
    // A and stage s+2's B are issued at the top of stage s; the barrier at its end waits for
    // everything but B(s+2) (issued last: vmcnt(GB)). A(s+1) refills the A buffer and B(s+2) the B
    // buffer stage s-1 was read from (every wave's reads of it completed before the last barrier).
    typedef V2Half<Cfg, QT, ABL> Half;
    auto abuf = [&](int s) { return lds + (s & 1) * Cfg::A_BYTES; };
    auto bbuf = [&](int s) { return lds + 2 * Cfg::A_BYTES + (s % 3) * Cfg::B_BYTES; };
    auto issue_a = [&](int s) { v2_dma<GA>(srcA, abuf(s), (ks0 + s) * Cfg::BKB, kbytes, wave, lane); };
    auto issue_b = [&](int s) { v2_dma<GB>(srcB, bbuf(s), (ks0 + s) * Cfg::BKB, kbytes, wave, lane); };
    auto hread = [&](Half& f, int s, int h) { f.read(abuf(s), bbuf(s), a_row, b_row, swz, g, h); };
    auto hmma = [&](const Half& f) { f.mma(acc); };
    auto sync_next = [&](int s) {  // stage s+1 landed for every wave
      if (s + 2 < nst) wait_vmcnt<GB>();
      else wait_vmcnt<0>();
      lds_barrier();
    };
    if (nst > 0) {
      Half fr;
      issue_a(0);
      issue_b(0);
      if (nst > 1) issue_b(1);
      sync_next(-1);
      if (wave >= Cfg::WM * Cfg::WN / 2) {
        for (int s = 0; s < nst; ++s) {
          if (s + 1 < nst) issue_a(s + 1);
          if (s + 2 < nst) issue_b(s + 2);
          if (s > 0) hmma(fr);
          hread(fr, s, 0);
          hmma(fr);
          hread(fr, s, 1);
          sync_next(s);
        }
        hmma(fr);
      } else {
        for (int s = 0; s < nst; ++s) {
          if (s + 1 < nst) issue_a(s + 1);
          if (s + 2 < nst) issue_b(s + 2);
          hread(fr, s, 0);
          hmma(fr);
          hread(fr, s, 1);
          hmma(fr);
          sync_next(s);
        }
      }
    }
    stash_scale();  // the rings are dead: the scale stash (past the epilogue image) is free
    if constexpr (qt_scaled(QT)) __syncthreads();
  } else if constexpr ((ABL & V2_STAGGER) != 0) {
    typedef V2Half<Cfg, QT, ABL> Half;
    auto hread = [&](Half& f, int buf, int h) {
      f.read(lds + buf * Cfg::STAGE_BYTES, lds + buf * Cfg::STAGE_BYTES + Cfg::A_BYTES, a_row, b_row, swz, g, h);
    };
    auto hmma = [&](const Half& f) { f.mma(acc); };
    auto stage_sync = [&](int) { __syncthreads(); };  // stage s+1 landed, buffer s&1 released
    if (nst > 0) {
      Half fr;  // one fragment set (the late schedule carries it across the barrier)
      issue(0, 0);
      stage_sync(-1);
      stash_scale();
      if (wave >= Cfg::WM * Cfg::WN / 2) {  // late: straight-line loop of its own
        for (int s = 0; s < nst; ++s) {
          if (s + 1 < nst) issue(s + 1, (s + 1) & 1);
          if (s > 0) hmma(fr);  // second half of stage s-1 (its buffer may be refilled now)
          hread(fr, s & 1, 0);
          hmma(fr);
          hread(fr, s & 1, 1);  // landed before the barrier below (it waits lgkmcnt(0))
          stage_sync(s);
        }
        hmma(fr);
      } else {
        for (int s = 0; s < nst; ++s) {
          if (s + 1 < nst) issue(s + 1, (s + 1) & 1);
          hread(fr, s & 1, 0);
          hmma(fr);
          hread(fr, s & 1, 1);
          hmma(fr);
          stage_sync(s);
        }
      }
    }
  } else if (nst > 0) {
    // ---- mainloop: stage s+1 in flight (LDS-DMA) while stage s is consumed ----
    issue(0, 0);
    __syncthreads();  // vmcnt(0) + barrier: stage 0 landed for every wave
    stash_scale();
    for (int s = 0; s < nst; ++s) {
      if (s + 1 < nst) issue(s + 1, (s + 1) & 1);
      compute(s & 1);
      if constexpr ((ABL & ABL_B_REGLOAD) != 0) {
#pragma unroll
        for (int j = 0; j < GB; ++j) asm volatile("" ::"v"(breg[j].x), "v"(breg[j].y), "v"(breg[j].z), "v"(breg[j].w));
      }
      __syncthreads();  // own LDS-DMA landed (vmcnt(0)); every wave done reading buffer s&1
    }
  }

  if ((ABL & V2_B3) == 0 && nst <= 0) {  // no mainloop barrier behind the stash
    stash_scale();
    __syncthreads();
  }
  if constexpr ((ABL & V2_TRACE) != 0 && (ABL & (V2_TRACE_PRO | V2_TRACE_DESC)) == 0) trace_mark(1);
  if (!splitk_reduce<Cfg::NT>(acc, sk, lds)) return;  // split-K: only the last slice writes C

  // ---- epilogue: per-wave LDS staging of the fp16 sub-tile, 16-B row stores ----
  // (B3: the lane decomposition is recomputed from an opaque copy of the thread id, so the
  // compiler does not keep it live — and spilled — across the 160-KiB mainloop)
  int etid = tid;
  if constexpr ((ABL & V2_B3) != 0) asm volatile("" : "+v"(etid));
  const int e_lane = etid & 63, e_r16 = e_lane & 15, e_g = e_lane >> 4;
  uint8_t* reg = lds + wave * (Cfg::WTM * Cfg::WTN * 2);
  const int mrow0 = m0 + wm * Cfg::WTM, ncol0 = n0 + wn * Cfg::WTN;
  // int paths: the tile's row / column scales were staged in LDS during the prologue
  const _Float16* sl = reinterpret_cast<const _Float16*>(lds + Cfg::LDS_BYTES);
  uint2 sbw[FN];
  if constexpr (qt_scaled(QT)) {
#pragma unroll
    for (int j = 0; j < FN; ++j) sbw[j] = *reinterpret_cast<const uint2*>(sl + 256 + wn * Cfg::WTN + j * 16 + 4 * e_g);
  }
  auto pack_frag = [&](int i, int j, _Float16 sai) {
    if constexpr (QT == QT_F16 || QT == QT_BF16) return pack4_f16(acc[i][j]);
    else if constexpr (QT == QT_F8) return scale_pack4f(acc[i][j], sai, sbw[j]);
    else return scale_pack4<(QT == QT_I4) ? 8 : 0>(acc[i][j], sai, sbw[j]);
  };
  auto pack_row = [&](int i) {  // fragment row i (16 rows of the wave's sub-tile) -> LDS
    const int ml = i * 16 + e_r16;
    _Float16 sai = 0;
    if constexpr (qt_scaled(QT)) sai = sl[wm * Cfg::WTM + ml];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 pk = pack_frag(i, j, sai);
      const int q = 2 * j + (e_g >> 1);
      *reinterpret_cast<uint2*>(reg + ml * 128 + ((q ^ (ml & 7)) << 4) + (e_g & 1) * 8) = pk;
    }
  };
  if constexpr (QT == QT_F16 || QT == QT_I8 || QT == QT_I4) {
    if ((mt.reserved2 & META_SILU) != 0) {
      // fused SiLU: fragments 2 jp (gate) and 2 jp + 1 (up) hold the same 16 output columns; the
      // wave's 32 output columns are staged as 64-B rows and stored 16 rows per instruction
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = i * 16 + e_r16;
        _Float16 sai = 0;
        if constexpr (qt_scaled(QT)) sai = sl[wm * Cfg::WTM + ml];
#pragma unroll
        for (int jp = 0; jp < FN / 2; ++jp) {
          const uint2 h = silu_mul4(pack_frag(i, 2 * jp, sai), pack_frag(i, 2 * jp + 1, sai));
          const int q = 2 * jp + (e_g >> 1);
          *reinterpret_cast<uint2*>(reg + ml * 64 + ((q ^ (ml & 3)) << 4) + (e_g & 1) * 8) = h;
        }
      }
      const int ocol0 = ncol0 / 2, NO = N / 2;
      _Float16* const obase = C + (int64_t)mrow0 * mt.ldc + ocol0;
      const bool onarrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;  // byte offsets < 2^30
#pragma unroll 4
      for (int it = 0; it < Cfg::WTM / 16; ++it) {
        const int row = it * 16 + (e_lane >> 2), q = e_lane & 3;
        const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 64 + ((q ^ (row & 3)) << 4));
        if (mrow0 + row < M && ocol0 + q * 8 < NO)
          store_c16<(ABL & V2_PLAINST) ? 0 : 16>(obase, (int64_t)row * mt.ldc + q * 8, onarrow, v);
      }
      return;
    }
  }
  _Float16* const cbase = C + (int64_t)mrow0 * mt.ldc + ncol0;  // wave-uniform
  const bool narrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;  // byte offsets < 2^30
  // (a wave reads back only its own region: LDS keeps one wave's accesses in order)
  auto store_rows = [&](int it) {  // rows [8 it, 8 it + 8) of the wave's sub-tile, 16 B per lane
    const int row = it * 8 + (e_lane >> 3), q = e_lane & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 128 + ((q ^ (row & 7)) << 4));
    const int m = mrow0 + row, n = ncol0 + q * 8;
    if constexpr ((ABL & ABL_NO_EPI) != 0) {
      asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    } else {
      if (m < M && n < N) store_c16<(ABL & V2_PLAINST) ? 0 : 16>(cbase, (int64_t)row * mt.ldc + q * 8, narrow, v);
    }
  };
  if constexpr ((ABL & V2_EPIPE) != 0) {
    // stores of fragment row i - 1 issued behind the LDS writes of row i: the first 2 KiB of the
    // wave's 16 KiB leave after one eighth of the pack VALU, the rest drain under the remaining rows
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      pack_row(i);
      if (i > 0) {
        store_rows(2 * i - 2);
        store_rows(2 * i - 1);
      }
    }
    store_rows(2 * FM - 2);
    store_rows(2 * FM - 1);
  } else {
#pragma unroll
    for (int i = 0; i < FM; ++i) pack_row(i);
#pragma unroll 4
    for (int it = 0; it < Cfg::WTM / 8; ++it) store_rows(it);
  }
}

// ============================================================================================
// w4a4 g128 (reference cta_gemm_w4a4g128, cta_gemm.cuh:610-772, Atom-style): per 128-K group an
// exact int32 dot product, folded into an f32 accumulator in group order,
//     out = fma(f32(acc_g), f32(fp16_rn(sa_g[m] * sb_g[n])), out),   C = fp16_rn(out)
// (`frag_out += T(acc) * T(sa * sb)`, mm_tile.cuh:490-493, which nvcc contracts to one FFMA).
// Scales: fp16 [K/128][M] and [K/128][N] (permute_scale, quantize.cuh:299-315; test.cu:283-313).
//
// MI355X layout: the v2 tiles (8 waves 2M x 4N; 256-row class with 128 x 64 wave tiles, 128-row
// class for a problem's last rows). The f32 fold accumulators live in registers for the whole
// tile, the int32 group accumulators only for two fragment rows at a time (row-pipelined fold,
// below), which is what lets the 128 x 64 wave tile fit without spills. One 128-B K stage = 256 int4 = two groups: MFMA steps 0-1 form group 2s, steps
// 2-3 group 2s+1, each group's first MFMA starting from a zero accumulator operand. The widened
// nibbles make acc = 256 * sum(a*b) (exact, |acc| < 2^22); the fold runs on that raw value and the
// store multiplies by 2^-8 — power-of-two scaling commutes with every rounding here (all partial
// values are multiples of 2^-16, far from f32 under/overflow), so the result is the reference's
// bit for bit, for 2.5 VALU per output per group (v_cvt_f32_i32, v_fma_mix_f32, half a
// v_pk_mul_f16). Group scales of stage s+1 are loaded (one or two halves per thread) before that
// stage's DMA, written to a 1.5-KiB LDS slot after stage s's MFMAs, and published by the stage
// barrier. Not split along K (an f32 partial sum would change the rounding order).
// ============================================================================================
__device__ __forceinline__ float fma_f32_f16lo(float a, uint32_t s, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(s), "v"(c));
  return d;
}
__device__ __forceinline__ float fma_f32_f16hi(float a, uint32_t s, float c) {
  float d;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(d) : "v"(a), "v"(s), "v"(c));
  return d;
}

template <class Cfg>
__device__ __forceinline__ void gg_tile_g128(const GGMeta& mt, const uint8_t* __restrict__ A,
                                             const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                             const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0, int n0,
                                             uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB;
  static_assert(Cfg::BM <= 256 && Cfg::BN == 256, "scale slot holds 256 rows / columns per group");
  constexpr int SCL = 2 * Cfg::STAGE_BYTES;  // LDS scale slots: [buf][sa 2 x 256 | sb 2 x 256] fp16
  constexpr int SCL_BYTES = 2048;
  static_assert(SCL + 2 * SCL_BYTES <= V2Cfg<256>::LDS_BYTES + V2_LDS_EXTRA, "scale slots must fit the v2 LDS image");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N, kbytes = mt.kbytes, ngroups = mt.reserved;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = (kbytes + Cfg::BKB - 1) / Cfg::BKB;

  const uint8_t* srcA[GA];
  const uint8_t* srcB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      srcA[j] = A + (int64_t)min(m0 + row, M - 1) * lda + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      srcB[j] = B + (int64_t)min(n0 + row, N - 1) * ldb + ((p ^ ((row >> 1) & 7)) << 4);
    }
  }
  auto issue = [&](int s, int buf) {
    uint8_t* As = lds + buf * Cfg::STAGE_BYTES;
    uint8_t* Bs = As + Cfg::A_BYTES;
    const int kb = s * Cfg::BKB;
    if (kb + Cfg::BKB <= kbytes) {
#pragma unroll
      for (int j = 0; j < GA; ++j) glds16(srcA[j] + kb, As + (wave * GA + j) * 1024);
#pragma unroll
      for (int j = 0; j < GB; ++j) glds16(srcB[j] + kb, Bs + (wave * GB + j) * 1024);
    } else {  // K tail: the second group of the last stage does not exist; its chunks load zeros
      const int rsub = lane >> 3, p = lane & 7;
      const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero16);
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int kc = (p ^ ((((wave * GA + j) * 8 + rsub) >> 1) & 7)) << 4;
        glds16(kb + kc < kbytes ? srcA[j] + kb : zero, As + (wave * GA + j) * 1024);
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int kc = (p ^ ((((wave * GB + j) * 8 + rsub) >> 1) & 7)) << 4;
        glds16(kb + kc < kbytes ? srcB[j] + kb : zero, Bs + (wave * GB + j) * 1024);
      }
    }
  };
  // group scales of stage s (groups 2s, 2s+1), two halves per thread: threads 0-255 the sa of tile
  // row tid (rows < BM), threads 256-511 the sb of tile column tid - 256
  uint32_t sc = 0;
  auto load_scales = [&](int s) {
    const int g0 = 2 * s;
    const bool two = g0 + 1 < ngroups;
    if (tid < 256) {
      if (tid < Cfg::BM) {
        const int64_t r = min(m0 + tid, M - 1);
        const uint32_t lo = __builtin_bit_cast(uint16_t, SA[(int64_t)g0 * M + r]);
        const uint32_t hi = two ? __builtin_bit_cast(uint16_t, SA[(int64_t)(g0 + 1) * M + r]) : 0u;
        sc = lo | (hi << 16);
      }
    } else {
      const int64_t n = min(n0 + tid - 256, N - 1);
      const uint32_t lo = __builtin_bit_cast(uint16_t, SB[(int64_t)g0 * N + n]);
      const uint32_t hi = two ? __builtin_bit_cast(uint16_t, SB[(int64_t)(g0 + 1) * N + n]) : 0u;
      sc = lo | (hi << 16);
    }
  };
  auto stash_scales = [&](int buf) {
    uint16_t* sl = reinterpret_cast<uint16_t*>(lds + SCL + buf * SCL_BYTES);
    if (tid >= 256 || tid < Cfg::BM) {
      const int c = tid < 256 ? tid : 512 + tid - 256;
      sl[c] = (uint16_t)sc;
      sl[c + 256] = (uint16_t)(sc >> 16);
    }
  };

  v4f out[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) out[i][j] = v4f{0, 0, 0, 0};

  const int swz = (r16 >> 1) & 7;
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u;
  const uint32_t b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  // fold of fragment row i: out += f32(acc) * f32(fp16_rn(sa * sb)), one rounding (v_fma_mix_f32)
  auto fold = [&](int i, const v4i (&acc)[FN], const uint2 (&sbw)[FN], _Float16 sai) {
    const h2_t sa2 = {sai, sai};
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint32_t s01 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw[j].x));
      const uint32_t s23 = __builtin_bit_cast(uint32_t, sa2 * __builtin_bit_cast(h2_t, sbw[j].y));
      out[i][j][0] = fma_f32_f16lo((float)acc[j][0], s01, out[i][j][0]);
      out[i][j][1] = fma_f32_f16hi((float)acc[j][1], s01, out[i][j][1]);
      out[i][j][2] = fma_f32_f16lo((float)acc[j][2], s23, out[i][j][2]);
      out[i][j][3] = fma_f32_f16hi((float)acc[j][3], s23, out[i][j][3]);
    }
  };
  // one group = two 64-element MFMA steps. Row-pipelined: the group's B fragments (both steps)
  // stay in registers, fragment row i's int32 accumulators are formed by 2 * FN MFMAs and folded
  // while row i+1's MFMAs run (two accumulator sets) — the fold's VALU sits beside the matrix
  // pipe's work instead of after all of it, and only 2 * FN int32 fragments are ever live.
  auto compute = [&](int buf, int s) {
    const uint8_t* As = lds + buf * Cfg::STAGE_BYTES + a_row;
    const uint8_t* Bs = lds + buf * Cfg::STAGE_BYTES + Cfg::A_BYTES + b_row;
    const _Float16* sl = reinterpret_cast<const _Float16*>(lds + SCL + buf * SCL_BYTES);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && 2 * s + 1 >= ngroups) break;  // K tail: no second group in this stage
      const uint32_t off0 = (uint32_t)(((4 * h + (g >> 1)) ^ swz) << 4) + (uint32_t)((g & 1) * 8);
      const uint32_t off1 = (uint32_t)(((4 * h + 2 + (g >> 1)) ^ swz) << 4) + (uint32_t)((g & 1) * 8);
      v4i b0[FN], b1[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        b0[j] = widen_i4(*reinterpret_cast<const v2i*>(Bs + j * 2048 + off0));
        b1[j] = widen_i4(*reinterpret_cast<const v2i*>(Bs + j * 2048 + off1));
      }
      const uint2* sbp = reinterpret_cast<const uint2*>(sl + 512 + h * 256 + wn * Cfg::WTN + 4 * g);
      uint2 sbw[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) sbw[j] = sbp[j * 4];
      const _Float16* sa = sl + h * 256 + wm * Cfg::WTM + r16;
      v4i acc0[FN], acc1[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        v4i (&acc)[FN] = (i & 1) ? acc1 : acc0;
        const v4i a0 = widen_i4(*reinterpret_cast<const v2i*>(As + i * 2048 + off0));
        const v4i a1 = widen_i4(*reinterpret_cast<const v2i*>(As + i * 2048 + off1));
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b0[j], a0, v4i{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b1[j], a1, acc[j], 0, 0, 0);
        if (i > 0) fold(i - 1, (i & 1) ? acc0 : acc1, sbw, sa[(i - 1) * 16]);
      }
      fold(FM - 1, ((FM - 1) & 1) ? acc1 : acc0, sbw, sa[(FM - 1) * 16]);
    }
  };

  if (nst > 0) {
    load_scales(0);
    issue(0, 0);
    stash_scales(0);  // waits for the scale loads only (issued before the DMA)
    __syncthreads();  // stage 0 and its scales visible
    for (int s = 0; s < nst; ++s) {
      if (s + 1 < nst) {
        load_scales(s + 1);  // before the DMA: the wait on them leaves the DMA in flight
        issue(s + 1, (s + 1) & 1);
      }
      compute(s & 1, s);
      if (s + 1 < nst) stash_scales((s + 1) & 1);  // slot last read by stage s-1 (before the last barrier)
      __syncthreads();
    }
  }

  // ---- epilogue (as gg_tile_v2): out * 2^-8 (exact) -> fp16, per-wave LDS staging, 16-B stores ----
  // (lane indices re-derived from an opaque copy of threadIdx.x: keeping the mainloop's copies live
  // across the K loop cost the 256-row body a VGPR spill)
  int etid = threadIdx.x;
  asm volatile("" : "+v"(etid));
  const int elane = etid & 63, er16 = elane & 15, eg = elane >> 4;
  uint8_t* reg = lds + wave * (Cfg::WTM * Cfg::WTN * 2);
  const int mrow0 = m0 + wm * Cfg::WTM, ncol0 = n0 + wn * Cfg::WTN;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = i * 16 + er16;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 pk = pack4_f16(out[i][j] * (1.0f / 256.0f));
      const int q = 2 * j + (eg >> 1);
      *reinterpret_cast<uint2*>(reg + ml * 128 + ((q ^ (ml & 7)) << 4) + (eg & 1) * 8) = pk;
    }
  }
  _Float16* const cbase = C + (int64_t)mrow0 * mt.ldc + ncol0;  // wave-uniform
  const bool narrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;  // byte offsets < 2^30
#pragma unroll 4
  for (int it = 0; it < Cfg::WTM / 8; ++it) {
    const int row = it * 8 + (elane >> 3), q = elane & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(reg + row * 128 + ((q ^ (row & 7)) << 4));
    const int m = mrow0 + row, n = ncol0 + q * 8;
    if (m < M && n < N) store_c16(cbase, (int64_t)row * mt.ldc + q * 8, narrow, v);
  }
}

// v2 fused kernel: qtype x height-class dispatch, uniform per workgroup.


// ============================================================================================
// v3: as v2 (8 waves 2M x 4N, BN = 256, height classes 256 / 128, LDS-DMA, swapped MFMA operands,
// LDS-staged epilogue) but K is staged 64 BYTES at a time through a 4-deep LDS ring with a
// prefetch distance of 3 stages: the DMAs of stages s+1 and s+2 stay in flight across the barrier
// of stage s (counted `s_waitcnt vmcnt(N)` + raw `s_barrier`, never vmcnt(0) in the loop).
//   LDS rows are 64 B (4 x 16-B chunks); chunk c of row r sits at c ^ T[(r >> 2) & 3],
//   T = {0, 2, 3, 1} — conflict-free for the 16-row ds_read_b128 (int8 / fp16) and ds_read_b64
//   (int4) fragment reads (exhaustive check over the gfx950 lane groups).
// Ring safety: stage s+3 is written into the buffer stage s-1 was read from; the barrier of
// iteration s follows every wave's compute(s-1) (its ds_reads are consumed by MFMAs before it).
// ============================================================================================
template <int BM_, int BN_ = 256, int WN_ = 4, int NBUF_ = 4, int DIST_ = 3>
struct V3Cfg {
  static constexpr int BM = BM_, BN = BN_, BKB = 64, NBUF = NBUF_, DIST = DIST_;
  static constexpr int WM = 2, WN = WN_, NT = WM * WN * 64, NWAVES = WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int A_BYTES = BM * BKB, B_BYTES = BN * BKB, STAGE_BYTES = A_BYTES + B_BYTES;
  // LDS-DMA wave-instructions per wave per stage (one covers 16 rows x 64 B)
  static constexpr int GA = BM / (16 * NWAVES), GB = BN / (16 * NWAVES);
  static constexpr int DMA_PER_STAGE = GA + GB;
  static constexpr int EPI_BYTES = WM * WN * WTM * WTN * 2;
  static constexpr int RING_BYTES = NBUF * STAGE_BYTES;
  static constexpr int LDS_BYTES = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  static_assert(WTN == 64 || WTN == 128, "epilogue stages 128-B or 256-B rows");
  static_assert(GA >= 1 && GB >= 1, "each wave issues at least one DMA per operand");
  static_assert(DIST < NBUF && DIST <= 4, "ring: stage s+DIST reuses the buffer of stage s-1 at most");
};

// buffer-form LDS-DMA of one 16-B chunk per lane (v3x): resource `rs`, lane offset `vo`, stage offset `so`
__device__ __forceinline__ __amdgpu_buffer_rsrc_t v3_rsrc(const uint8_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void v3_bdma(__amdgpu_buffer_rsrc_t rs, uint8_t* dst, uint32_t vo, int so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)dst, 16, vo, so, 0, 0);
}

__device__ __forceinline__ int swz64(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }  // T = {0,2,3,1}


// Epilogue shared by v3 / v4: dequant (int paths) + fp16 rounding, per-wave LDS staging of the
// WTM x WTN fp16 sub-tile in XOR-swizzled 16-B chunks, then 16-B row stores (coalesced along N).
// Needs WTM * WTN * 2 bytes of LDS per wave at `lds` (the drained ring).
// SILU: compile the fused SiLU epilogue in (v3 tiles; the weight-only tiles, which never carry the
// flag, leave it out — its code cost their 3-WG/CU build a spill)
template <class Cfg, int QT, bool SILU = true>
__device__ __forceinline__ void epilogue_v3(const GGMeta& mt, typename AccT<QT>::type (&acc)[Cfg::FM][Cfg::FN],
                                            const _Float16* __restrict__ SA, const _Float16* __restrict__ SB,
                                            _Float16* __restrict__ C, int m0, int n0, uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N;
  constexpr int RB = Cfg::WTN * 2, CPR = RB / 16;  // staged row bytes, 16-B chunks per row
  uint8_t* reg = lds + wave * (Cfg::WTM * Cfg::WTN * 2);
  const int mrow0 = m0 + wm * Cfg::WTM, ncol0 = n0 + wn * Cfg::WTN;
  // column scales: one 8-B load per 4 columns (N % 8 == 0 keeps the clamped address 8-B
  // aligned); the row scale is loaded per fragment row -> 2*FN + 1 live registers, not 5*FN
  uint2 sbw[FN];
  if constexpr (QT != QT_F16) {
#pragma unroll
    for (int j = 0; j < FN; ++j) sbw[j] = *reinterpret_cast<const uint2*>(SB + min(ncol0 + j * 16 + 4 * g, N - 4));
  }
  auto pack_frag = [&](int i, int j, _Float16 sai) {
    if constexpr (QT == QT_F16) return pack4_f16(acc[i][j]);
    else if constexpr (QT == QT_I4F6) return scale_pack4f(acc[i][j], sai, sbw[j]);
    else return scale_pack4<(QT == QT_I4) ? 8 : 0>(acc[i][j], sai, sbw[j]);
  };
  if constexpr (SILU && (QT == QT_F16 || QT == QT_I8 || QT == QT_I4)) {
    if ((mt.reserved2 & META_SILU) != 0) {  // fused SiLU (as gg_tile_v2): rows of WTN / 2 outputs
      constexpr int ORB = Cfg::WTN, OCPR = ORB / 16;  // staged output row bytes, 16-B chunks per row
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = i * 16 + r16;
        _Float16 sai = 0;
        if constexpr (QT != QT_F16) sai = SA[min(mrow0 + ml, M - 1)];
#pragma unroll
        for (int jp = 0; jp < FN / 2; ++jp) {
          const uint2 h = silu_mul4(pack_frag(i, 2 * jp, sai), pack_frag(i, 2 * jp + 1, sai));
          const int q = 2 * jp + (g >> 1);
          *reinterpret_cast<uint2*>(reg + ml * ORB + ((q ^ (ml & (OCPR - 1))) << 4) + (g & 1) * 8) = h;
        }
      }
      constexpr int ORPI = 64 / OCPR;
      const int ocol0 = ncol0 / 2, NO = N / 2;
      _Float16* const obase = C + (int64_t)mrow0 * mt.ldc + ocol0;
      const bool onarrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;
#pragma unroll 4
      for (int it = 0; it < Cfg::WTM / ORPI; ++it) {
        const int row = it * ORPI + lane / OCPR, q = lane % OCPR;
        const uint4 v = *reinterpret_cast<const uint4*>(reg + row * ORB + ((q ^ (row & (OCPR - 1))) << 4));
        if (mrow0 + row < M && ocol0 + q * 8 < NO) store_c16(obase, (int64_t)row * mt.ldc + q * 8, onarrow, v);
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = i * 16 + r16;
    _Float16 sai = 0;
    if constexpr (QT != QT_F16) sai = SA[min(mrow0 + ml, M - 1)];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 pk = pack_frag(i, j, sai);  // (QT_I4F6: the f32 acc is the int32 sum)
      const int q = 2 * j + (g >> 1);
      *reinterpret_cast<uint2*>(reg + ml * RB + ((q ^ (ml & (CPR - 1))) << 4) + (g & 1) * 8) = pk;
    }
  }
  constexpr int RPI = 64 / CPR;  // staged rows per wave-instruction
  _Float16* const cbase = C + (int64_t)mrow0 * mt.ldc + ncol0;  // wave-uniform
  const bool narrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;  // byte offsets < 2^30
#pragma unroll 4
  for (int it = 0; it < Cfg::WTM / RPI; ++it) {
    const int row = it * RPI + lane / CPR, q = lane % CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(reg + row * RB + ((q ^ (row & (CPR - 1))) << 4));
    const int m = mrow0 + row, n = ncol0 + q * 8;
    if (m < M && n < N) store_c16(cbase, (int64_t)row * mt.ldc + q * 8, narrow, v);
  }
}

// OPT (v3x, lab): 1 = buffer-form LDS-DMA (per-tile buffer resources, fixed 32-bit lane offsets,
// the stage's K offset in soffset; K-tail chunks past num_records read as zeros) issued one piece
// per k MFMAs through the steady-state stage (sched_group_barrier), as v2x does for v2
template <class Cfg, int QT, int OPT = 0>
__device__ __forceinline__ void gg_tile_v3(const GGMeta& mt, const uint8_t* __restrict__ A,
                                           const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                           const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0, int n0,
                                           uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB, DPS = Cfg::DMA_PER_STAGE;
  typedef typename AccT<QT>::type acc_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N, kbytes = mt.kbytes;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = (kbytes + Cfg::BKB - 1) / Cfg::BKB;

  // per-lane DMA sources: one wave-instruction = 16 rows x 64 B; lane -> (row r0 + lane/4, slot lane%4)
  const uint8_t* srcA[GA];
  const uint8_t* srcB[GB];
  int kcA[GA], kcB[GB];  // logical chunk byte offset of this lane (for the K tail)
  {
    const int rsub = lane >> 2, p = lane & 3;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 16 + rsub;
      kcA[j] = (p ^ swz64(row)) << 4;
      srcA[j] = A + (int64_t)min(m0 + row, M - 1) * lda + kcA[j];
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 16 + rsub;
      kcB[j] = (p ^ swz64(row)) << 4;
      srcB[j] = B + (int64_t)min(n0 + row, N - 1) * ldb + kcB[j];
    }
  }
  const uint8_t* zero = reinterpret_cast<const uint8_t*>(g_zero16);
  auto issue = [&](int s) {
    uint8_t* As = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES;
    uint8_t* Bs = As + Cfg::A_BYTES;
    const int kb = s * Cfg::BKB;
    if (kb + Cfg::BKB <= kbytes) {
#pragma unroll
      for (int j = 0; j < GA; ++j) glds16(srcA[j] + kb, As + (wave * GA + j) * 1024);
#pragma unroll
      for (int j = 0; j < GB; ++j) glds16(srcB[j] + kb, Bs + (wave * GB + j) * 1024);
    } else {  // K tail: lanes past K load 16 zero bytes
#pragma unroll
      for (int j = 0; j < GA; ++j) glds16(kb + kcA[j] < kbytes ? srcA[j] + kb : zero, As + (wave * GA + j) * 1024);
#pragma unroll
      for (int j = 0; j < GB; ++j) glds16(kb + kcB[j] < kbytes ? srcB[j] + kb : zero, Bs + (wave * GB + j) * 1024);
    }
  };

  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  const int sw = swz64(r16);
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 64u;
  const uint32_t b_row = (uint32_t)(wn * Cfg::WTN + r16) * 64u;
  auto compute = [&](int s) {
    const uint8_t* As = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES + a_row;
    const uint8_t* Bs = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES + Cfg::A_BYTES + b_row;
    if constexpr (QT == QT_I4) {
      // lane group g reads chunk g ^ sw of the 64-B row (16 B = 32 nibbles, ds_read_b128 as the int8
      // path: conflict-free under T) and runs two MFMA K steps on its 8-B halves; the same K map for
      // A and B (V2Half). Round 4 read 8 B per step, paired by hipcc into ds_read2st64_b64: PMC had
      // SQ_LDS_BANK_CONFLICT at 49 % of SQ_LDS_IDX_ACTIVE on the w4a4 layer
      const uint32_t off = (uint32_t)((g ^ sw) << 4);
      v4i braw[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) braw[j] = *reinterpret_cast<const v4i*>(Bs + j * 1024 + off);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        v4i b[FN];  // B widened once per step, A per fragment row
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = widen_i4(v2i{braw[j][2 * st], braw[j][2 * st + 1]});
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const v4i araw = *reinterpret_cast<const v4i*>(As + i * 1024 + off);
          const v4i a = widen_i4(v2i{araw[2 * st], araw[2 * st + 1]});
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a, acc[i][j], 0, 0, 0);
        }
      }
    } else {
      const uint32_t off = (uint32_t)((g ^ sw) << 4);
      if constexpr (QT == QT_I8) {
        v4i a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v4i*>(As + i * 1024 + off);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v4i*>(Bs + j * 1024 + off);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[j], a[i], acc[i][j], 0, 0, 0);
      } else {
        v8h a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const v8h*>(As + i * 1024 + off);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const v8h*>(Bs + j * 1024 + off);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
    }
  };

  if constexpr ((OPT & 1) != 0) {
    const __amdgpu_buffer_rsrc_t rsA = v3_rsrc(A + (int64_t)m0 * lda);
    const __amdgpu_buffer_rsrc_t rsB = v3_rsrc(B + (int64_t)n0 * ldb);
    uint32_t voA[GA], voB[GB];
    {
      const int rsub = lane >> 2;
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int row = (wave * GA + j) * 16 + rsub;
        voA[j] = (uint32_t)((min(m0 + row, M - 1) - m0) * lda) + kcA[j];
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int row = (wave * GB + j) * 16 + rsub;
        voB[j] = (uint32_t)((min(n0 + row, N - 1) - n0) * ldb) + kcB[j];
      }
    }
    auto bissue = [&](int s, bool full) {
      uint8_t* As = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES;
      uint8_t* Bs = As + Cfg::A_BYTES;
      const int kb = s * Cfg::BKB;
#pragma unroll
      for (int j = 0; j < GA; ++j)
        v3_bdma(rsA, As + (wave * GA + j) * 1024, full || kb + kcA[j] < kbytes ? voA[j] : 0x80000000u, kb);
#pragma unroll
      for (int j = 0; j < GB; ++j)
        v3_bdma(rsB, Bs + (wave * GB + j) * 1024, full || kb + kcB[j] < kbytes ? voB[j] : 0x80000000u, kb);
    };
    const int nfull = (nst * Cfg::BKB > kbytes) ? nst - 1 : nst;  // stages [0, nfull) have no K tail
#pragma unroll
    for (int p = 0; p < Cfg::DIST; ++p)
      if (p < nst) bissue(p, p < nfull);
    constexpr int NM = (QT == QT_I4 ? 2 : 1) * FM * FN;  // MFMAs per stage
    constexpr int KS = NM / DPS > 0 ? NM / DPS : 1;
    int s = 0;
    // steady state: stage s + DIST is full and exists; one basic block per stage
    for (; s + Cfg::DIST < nfull; ++s) {
      wait_vmcnt<(Cfg::DIST - 1) * DPS>();
      lds_barrier();
      bissue(s + Cfg::DIST, true);
      compute(s);
#pragma unroll
      for (int q = 0; q < DPS; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    for (; s < nst; ++s) {
      const int later = min(Cfg::DIST - 1, nst - 1 - s);
      if (later >= 3) wait_vmcnt<(Cfg::DIST >= 4 ? 3 : 2) * DPS>();
      else if (later == 2) wait_vmcnt<2 * DPS>();
      else if (later == 1) wait_vmcnt<DPS>();
      else wait_vmcnt<0>();
      lds_barrier();
      if (s + Cfg::DIST < nst) bissue(s + Cfg::DIST, s + Cfg::DIST < nfull);
      compute(s);
    }
    wait_vmcnt<0>();
    lds_barrier();  // ring -> epilogue staging
    epilogue_v3<Cfg, QT>(mt, acc, SA, SB, C, m0, n0, lds);
    return;
  }

  // ---- mainloop: 4-deep ring, 3 stages in flight ----
#pragma unroll
  for (int p = 0; p < Cfg::DIST; ++p)
    if (p < nst) issue(p);
  for (int s = 0; s < nst; ++s) {
    const int later = min(Cfg::DIST - 1, nst - 1 - s);  // stages issued after s so far
    if (later >= 3) wait_vmcnt<(Cfg::DIST >= 4 ? 3 : 2) * DPS>();
    else if (later == 2) wait_vmcnt<2 * DPS>();
    else if (later == 1) wait_vmcnt<DPS>();
    else wait_vmcnt<0>();
    lds_barrier();  // stage s landed for every wave; every wave is done with buffer (s-1)%4
    if (s + Cfg::DIST < nst) issue(s + Cfg::DIST);
    compute(s);
  }
  wait_vmcnt<0>();
  lds_barrier();  // ring -> epilogue staging

  epilogue_v3<Cfg, QT>(mt, acc, SA, SB, C, m0, n0, lds);
}

// QM = set of quant types compiled in (bit 1 << QType, chosen by the plan): a single-type launch
// carries one tile body, not three
// OPT & 4: one workgroup per CU, one wave per SIMD (512 registers: the accumulators of a 128 x 128
// wave tile live in AGPRs) — the 4-wave 256 x 256 tile widens each int4 fragment for 8 MFMAs, not 4
template <int BN, int WN, int NBUF, int DIST, int QM, int OPT = 0>
__global__ __launch_bounds__(128 * WN, (OPT & 4) ? 1 : 2) void gg_v3_kernel(GGArgs args) {  // 2 waves/SIMD: <= 256 VGPRs
  typedef V3Cfg<256, BN, WN, NBUF, DIST> CT;
  typedef V3Cfg<128, BN, WN, NBUF, DIST> CS;
  __shared__ __attribute__((aligned(16))) uint8_t lds[CT::LDS_BYTES];
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const GGMeta mt = args.meta[td.prob];
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[td.prob]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[td.prob]);
  const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
  const _Float16* SB = static_cast<const _Float16*>(args.ptr_SB[td.prob]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[td.prob]);
  const bool tall = td.cls == 0;
  if ((QM & (1 << QT_I8)) && mt.qtype == QT_I8) {
    if (tall) gg_tile_v3<CT, QT_I8, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
    else gg_tile_v3<CS, QT_I8, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
  } else if ((QM & (1 << QT_I4)) && mt.qtype == QT_I4) {
    if (tall) gg_tile_v3<CT, QT_I4, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
    else gg_tile_v3<CS, QT_I4, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
  } else if ((QM & (1 << QT_F16)) && mt.qtype == QT_F16) {
    if (tall) gg_tile_v3<CT, QT_F16, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
    else gg_tile_v3<CS, QT_F16, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
  }
}



// ============================================================================================
// Weight-only WxA16 (w4a16 / w8a16, any group size that is a multiple of 64 or per-channel,
// sym or asym): A fp16, B quantised codes dequantised in registers, fp16 MFMA, f32 accumulate.
// Reference arithmetic (cta_gemm.cuh:112-286, Converter::dequant_frag quantize.cuh:146-213):
// b = fp16(fma(u - off, scale, zp)) — one fp16 rounding, as the reference's __hfma2.
//   * a stage is 64 K ELEMENTS: A as the fp16 v2 path (rows of 128 B, same swizzle and fragment
//     reads), B rows of 64 * BITS / 8 bytes in the repacked layout of include/mxmoe_gg.h, so one
//     ds_read_b64 (4-bit) / ds_read_b128 (8-bit) gives a lane its 8 codes of both K halves;
//   * dequant: v_perm into 0x6400|u (= 1024 + u, exact fp16), v_pk_add_f16 -(1024 + off) (exact),
//     v_pk_fma_f16 with (scale, scale), (zp, zp);
//   * scale / zp (reference permute_scale layout [G][N] or [G][N][2]) per lane column, reloaded
//     when the stage enters a new group.
// ============================================================================================
// WM_ = waves along M: 2 for 256-row tiles; 1 for the 128 / 64-row classes, so that each B
// fragment is dequantised by exactly one wave and reused over all its 4-8 A fragments (with 2 x 4
// waves and 32-row wave tiles the dequant VALU outweighed the MFMAs 11:1 at small batch)
template <int BM_, int WM_ = 2, int LDSB_ = V2Cfg<256>::LDS_BYTES>
struct WoCfg {
  static constexpr int BM = BM_, BN = 256, NT = 512, KS = 64;  // KS: K elements per stage
  static constexpr int WM = WM_, WN = 8 / WM_;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int A_BYTES = BM * 128, B_BYTES_MAX = BN * KS;  // B sized for 8-bit codes
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES_MAX;
  static constexpr int GA = BM / 64;
  // LDS ring: as many stages as the kernel's 128-KiB image holds (2 at 256 rows, 4 at 128, 8 at 64
  // rows with 4-bit codes), all but one in flight — small tiles have little MFMA work per stage, so
  // they need the deeper prefetch to cover the load latency
  template <int BITS>
  static constexpr int stage_bytes() { return A_BYTES + BN * KS * BITS / 8; }
  template <int BITS>
  static constexpr int nbuf() {
    return LDSB_ / stage_bytes<BITS>() > 8 ? 8 : LDSB_ / stage_bytes<BITS>();
  }
  static constexpr int LDSB = LDSB_;
  static_assert(2 * STAGE_BYTES <= LDSB_, "two stages must fit the LDS image");
  static_assert(WM * WN * WTM * WTN * 2 <= LDSB_, "the epilogue's staged tile must fit the LDS image");
};

__device__ __forceinline__ uint32_t wo_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// 8 codes (K ascending) -> 8 fp16 dequantised values
// Register constants of the code -> fp16 step: with WO_ANDOR the tile makes them opaque (asm) so
// they stay in registers — gfx950's VOP3 takes no literal, so with literal constants the compiler
// splits v_and_or_b32 into v_and_b32 + v_or_b32 and keeps v_perm_b32 + v_or_b32 for 8-bit codes
struct WoK {
  uint32_t magic = 0x64006400u;  // fp16 1024 in both halves
  uint32_t mask4 = 0x000F000Fu, mask2 = 0x00030003u;
  uint32_t hi8 = 0x64646464u;   // 8-bit codes: v_perm_b32 takes the 0x64 bytes from here
  bool perm8 = false;           // 8-bit: one v_perm_b32 per pair (sel bytes 4 -> hi8)
  // nibpos (WO_NIBPOS): a code is read where it sits — the fp16 whose exponent puts the code's
  // lowest bit at weight 1 (bits 0 / 2 / 4 / 6: 1024 / 256 / 64 / 16 + u, exact), so a 4-bit word
  // needs one shift (by 8) instead of three and a 2-bit word none; the subtrahend per position
  // is -(base + off) (moffq), still exact, so fma(x, s, z) rounds as before
  bool nibpos = false;
  uint32_t nmask[4] = {0x000F000Fu, 0x00F000F0u, 0, 0};     // 4-bit: [0] bits 0-3, [1] bits 4-7
  uint32_t nmagic[4] = {0x64006400u, 0x54005400u, 0, 0};    // 1024, 64 (2-bit: 1024, 256, 64, 16)
  uint32_t moffq[4] = {0, 0, 0, 0};
};

template <int BITS>
__device__ __forceinline__ v8h wo_dequant(const uint32_t* w, uint32_t moff2, uint32_t s2, uint32_t z2,
                                          const WoK& k = WoK()) {
  uint32_t d[4];
  if constexpr (BITS == 4) {
    // repacked order: codes 2q, 2q+1 at bits 4q and 16 + 4q -> one v_and_or_b32 per fp16 pair
    if (k.nibpos) {
      const uint32_t w8 = w[0] >> 8;
      d[0] = (w[0] & k.nmask[0]) | k.nmagic[0];
      d[1] = (w[0] & k.nmask[1]) | k.nmagic[1];
      d[2] = (w8 & k.nmask[0]) | k.nmagic[0];
      d[3] = (w8 & k.nmask[1]) | k.nmagic[1];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = ((w[0] >> (4 * q)) & k.mask4) | k.magic;
    }
  } else if constexpr (BITS == 2) {
    // w[0] = the unit's 32-bit word pre-shifted by 8 * kc: codes 2q, 2q+1 at bits 2q and 16 + 2q
    if (k.nibpos) {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = (w[0] & k.nmask[q]) | k.nmagic[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = ((w[0] >> (2 * q)) & k.mask2) | k.magic;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // bytes 2q, 2q+1 of the 8 codes
      const uint32_t src = w[q >> 1];
      if (k.perm8) {
        d[q] = wo_perm(k.hi8, src, (q & 1) ? 0x04030402u : 0x04010400u);
      } else {
        const uint32_t sel = (q & 1) ? 0x0c030c02u : 0x0c010c00u;
        d[q] = wo_perm(0, src, sel) | 0x64006400u;
      }
    }
  }
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  v8h out;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t mo = (BITS != 8 && k.nibpos) ? k.moffq[q] : moff2;
    h2 x = __builtin_bit_cast(h2, d[q]) + __builtin_bit_cast(h2, mo);  // exact: u - off
    x = __builtin_elementwise_fma(x, __builtin_bit_cast(h2, s2), __builtin_bit_cast(h2, z2));
    out[2 * q] = x[0];
    out[2 * q + 1] = x[1];
  }
  return out;
}

template <class Cfg, int BITS, int WABL = 0>
__device__ __forceinline__ void gg_tile_wo(const GGMeta& mt, const uint8_t* __restrict__ A,
                                           const uint8_t* __restrict__ B, const _Float16* __restrict__ SB,
                                           _Float16* __restrict__ C, int m0, int n0, uint8_t* lds, const SplitK& sk) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA;
  constexpr int RB = Cfg::KS * BITS / 8;        // B bytes per row per stage
  // B DMA granule per lane: 16 B, or 4 B for 2-bit codes (16-B rows: 4 lanes per row, so every
  // wave still issues whole instructions and the vmcnt bookkeeping stays uniform)
  constexpr int GRAN = BITS == 2 ? 4 : 16;
  constexpr int LPR = RB / GRAN, RPI = 64 / LPR;  // lanes per B row, B rows per wave-instruction
  // B chunk swizzle: the 16-B chunk c of tile row n sits in LDS slot c ^ ((n >> RSH) & (LPR - 1)),
  // RSH = log2(rows per 256-B bank window); rows n, n + 256 / RB then hit different banks
  constexpr int RSH = BITS == 4 ? 3 : 2;
  constexpr int GBW = Cfg::BN / RPI / 8;        // B DMA instructions per wave per stage
  constexpr int SB_ = Cfg::template stage_bytes<BITS>(), NBUF = Cfg::template nbuf<BITS>(), DIST = NBUF - 1;
  constexpr int DPS = GA + GBW;  // LDS-DMA instructions per wave per stage
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = sk.nst, ks0 = sk.ks0;  // 64-K stages [ks0, ks0 + nst) of this tile
  const int gstages = mt.reserved;  // stages per scale group (>= nst: one group)
  const bool sym = (mt.reserved2 & 1) != 0;  // (bit META_SILU: the fused SiLU epilogue)

  const uint8_t* srcA[GA];
  const uint8_t* srcB[GBW];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      srcA[j] = A + (int64_t)min(m0 + row, M - 1) * lda + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GBW; ++j) {
      const int row = (wave * GBW + j) * RPI + lane / LPR;
      // source chunk for this LDS slot (2-bit: 4-B granules, rows unswizzled)
      const int chunk = BITS == 2 ? lane % LPR : (lane % LPR) ^ ((row >> RSH) & (LPR - 1));
      srcB[j] = B + (int64_t)min(n0 + row, N - 1) * ldb + chunk * GRAN;
      if constexpr ((WABL & ABL_WO_BTILED) != 0)
        srcB[j] = B + (int64_t)(n0 / Cfg::BN) * (mt.K / 64) * (Cfg::BN * RB) + row * RB + chunk * GRAN;
    }
  }
  // WO_ADEAD (64-row tiles: one A piece of 8 rows per wave): a wave whose 8 A rows all lie past M
  // issues no A piece — those LDS rows feed only output rows that are never stored — and counts
  // GBW pieces per stage in its waits
  static_assert((WABL & WO_ADEAD) == 0 || ((WABL & WO_SPLIT) != 0 && (WABL & WO_SCLATE) != 0),
                "the per-wave piece count is only honoured by the split WO_SCLATE loop");
  const bool a_live = (WABL & WO_ADEAD) == 0 || GA != 1 || wave * 8 < M - m0;
  // WO_BUF: buffer-form LDS-DMA (as v2x's V2_BUF): the tile's A / B bases in SGPR resources, a fixed
  // 32-bit lane offset, the stage's K offset in soffset — no 64-bit address add per piece
  constexpr bool kBuf = (WABL & WO_BUF) != 0 && (WABL & ABL_WO_BTILED) == 0;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(A) + (int64_t)m0 * lda, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(B) + (int64_t)n0 * ldb, (short)0, 0x7fffffff, 0x00020000);
  uint32_t voA[GA], voB[GBW];
  if constexpr (kBuf) {
#pragma unroll
    for (int j = 0; j < GA; ++j) voA[j] = (uint32_t)(srcA[j] - (A + (int64_t)m0 * lda));
#pragma unroll
    for (int j = 0; j < GBW; ++j) voB[j] = (uint32_t)(srcB[j] - (B + (int64_t)n0 * ldb));
  }
  auto issue = [&](int s, int buf) {
    if constexpr ((WABL & ABL_WO_NODMA) != 0) {
      if (s >= NBUF) return;
    }
    uint8_t* As = lds + buf * SB_;
    uint8_t* Bs = As + Cfg::A_BYTES;
    const int64_t boff = (WABL & ABL_WO_BTILED) ? (int64_t)(ks0 + s) * (Cfg::BN * RB) : (int64_t)(ks0 + s) * RB;
    if (a_live) {
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        if constexpr (kBuf)
          bdma16(rsA, As + (wave * GA + j) * 1024, voA[j], (ks0 + s) * 128);
        else
          glds16(srcA[j] + (ks0 + s) * 128, As + (wave * GA + j) * 1024);
      }
    }
#pragma unroll
    for (int j = 0; j < GBW; ++j) {
      if constexpr (kBuf && BITS == 2)
        bdma4(rsB, Bs + (wave * GBW + j) * 256, voB[j], (int)boff);
      else if constexpr (kBuf)
        bdma16(rsB, Bs + (wave * GBW + j) * 1024, voB[j], (int)boff);
      else if constexpr (BITS == 2)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(srcB[j] + boff), (lds_void_t*)(Bs + (wave * GBW + j) * 256), 4, 0, 0);
      else
        glds16(srcB[j] + boff, Bs + (wave * GBW + j) * 1024);
    }
  };

  // per-lane columns and their scale / zp pairs (packed (x, x) halves for v_pk_fma_f16)
  const int ncol0 = n0 + wn * Cfg::WTN;
  // fp16 -(1024 + off) = 0xE400 | off: sym off = 7 (4-bit) / 127 (8-bit), asym 0
  const uint32_t moff2 = sym ? (BITS == 4 ? 0xE407E407u : BITS == 2 ? 0xE401E401u : 0xE47FE47Fu) : 0xE400E400u;
  uint32_t s2[FN], z2[FN], s2n[FN], z2n[FN];  // current group, next group (prefetched)
  WoK wok;
  if constexpr ((WABL & WO_NIBPOS) != 0 && BITS != 8) {
    wok.nibpos = true;
    const int off = sym ? (BITS == 4 ? 7 : 1) : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int base = BITS == 4 ? ((q & 1) ? 64 : 1024) : (1024 >> (2 * q));  // 2-bit: 1024, 256, 64, 16
      if constexpr (BITS == 2) {
        wok.nmask[q] = 0x00030003u << (2 * q);
        wok.nmagic[q] = q == 0 ? 0x64006400u : q == 1 ? 0x5C005C00u : q == 2 ? 0x54005400u : 0x4C004C00u;
      }
      const uint32_t h = __builtin_bit_cast(uint16_t, (_Float16)(-(float)(base + off)));
      wok.moffq[q] = h | (h << 16);
    }
  }
  if constexpr ((WABL & WO_ANDOR) != 0) {
    wok.perm8 = true;
    if constexpr (BITS == 8) asm volatile("" : "+v"(wok.hi8));
    else if constexpr ((WABL & WO_NIBPOS) != 0 && BITS == 4)
      asm volatile("" : "+v"(wok.nmagic[0]), "+v"(wok.nmagic[1]), "+s"(wok.nmask[0]), "+s"(wok.nmask[1]));
    else if constexpr ((WABL & WO_NIBPOS) != 0 && BITS == 2)
      asm volatile("" : "+v"(wok.nmagic[0]), "+v"(wok.nmagic[1]), "+v"(wok.nmagic[2]), "+v"(wok.nmagic[3]),
                   "+s"(wok.nmask[0]), "+s"(wok.nmask[1]), "+s"(wok.nmask[2]), "+s"(wok.nmask[3]));
    else asm volatile("" : "+v"(wok.magic), "+s"(wok.mask4), "+s"(wok.mask2));
  }
  auto load_scales = [&](int grp, uint32_t (&so)[FN], uint32_t (&zo)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = min(ncol0 + j * 16 + r16, N - 1);
      if (sym) {
        const uint32_t s = __builtin_bit_cast(uint16_t, SB[(int64_t)grp * N + n]);
        so[j] = s | (s << 16);
        zo[j] = 0;
      } else {
        const uint32_t sz = *reinterpret_cast<const uint32_t*>(SB + ((int64_t)grp * N + n) * 2);
        so[j] = (sz & 0xFFFFu) * 0x10001u;
        zo[j] = (sz >> 16) * 0x10001u;
      }
    }
  };

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0, 0, 0, 0};

  const int swz = (r16 >> 1) & 7;
  // WO_MSKIP: the wave's 16-row blocks holding a row < M (small batches: ~35-row experts on 64-row tiles)
  const int nfm = __builtin_amdgcn_readfirstlane(min(FM, max(1, (M - m0 - wm * Cfg::WTM + 15) / 16)));
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u;
  const uint32_t b_row = (uint32_t)(wn * Cfg::WTN + r16) * RB;
  // rows of a B fragment are base + r16 with base % 16 == 0, so the swizzle depends on r16 only
  const int bsw = (r16 >> RSH) & (LPR - 1);
  auto compute = [&](int buf) {
    const uint8_t* As = lds + buf * SB_ + a_row;
    const uint8_t* Bs = lds + buf * SB_ + Cfg::A_BYTES + b_row;
    uint32_t raw[FN][2];  // 4-bit: the codes of both K halves (one 8-B read); 8-bit: one K half
    if constexpr (BITS == 2) {  // 2-bit: both K halves in one 4-B word (unit g of the 16-B row)
#pragma unroll
      for (int j = 0; j < FN; ++j) raw[j][0] = *reinterpret_cast<const uint32_t*>(Bs + j * 16 * RB + g * 4);
    }
    if constexpr (BITS == 4) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const uint2 v = *reinterpret_cast<const uint2*>(Bs + j * 16 * RB + (((g >> 1) ^ bsw) << 4) + (g & 1) * 8);
        raw[j][0] = v.x;
        raw[j][1] = v.y;
      }
    }
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const uint32_t off = (uint32_t)(((kc * 4 + g) ^ swz) << 4);
      v8h b[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if constexpr (BITS == 2) {
          const uint32_t w = raw[j][0] >> (8 * kc);
          b[j] = wo_dequant<2>(&w, moff2, s2[j], z2[j], wok);
        } else if constexpr (BITS == 4) {
          b[j] = wo_dequant<4>(&raw[j][kc], moff2, s2[j], z2[j], wok);
        } else {
          const uint2 v = *reinterpret_cast<const uint2*>(Bs + j * 16 * RB + ((g ^ bsw) << 4) + kc * 8);
          raw[j][0] = v.x;
          raw[j][1] = v.y;
          b[j] = wo_dequant<8>(raw[j], moff2, s2[j], z2[j], wok);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        // row block wholly past M: a uniform test per block (MEASURED NEGATIVE, round 4: one loop
        // copy per row-block count, NF = 1..4, was as fast on gate_up and 9-17 % slower on the
        // down calls, profiles/r04/wo/wo_g)
        if constexpr ((WABL & WO_MSKIP) != 0) {
          if (i > 0 && i >= nfm) break;
        }
        const v8h a = *reinterpret_cast<const v8h*>(As + i * 2048 + off);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a, acc[i][j], 0, 0, 0);
      }
    }
  };

  // wait until stage t's LDS-DMA (this wave's) has landed, `later` stages having been issued after it
  auto wait_stage_n = [&](int later, auto dps_c) {  // DPS_: pieces per stage of this wave
    constexpr int DPS_ = decltype(dps_c)::value;
    if constexpr (DIST >= 7) if (later >= 6) { wait_vmcnt<6 * DPS_>(); return; }
    if constexpr (DIST >= 6) if (later == 5) { wait_vmcnt<5 * DPS_>(); return; }
    if constexpr (DIST >= 5) if (later == 4) { wait_vmcnt<4 * DPS_>(); return; }
    if constexpr (DIST >= 4) if (later == 3) { wait_vmcnt<3 * DPS_>(); return; }
    if constexpr (DIST >= 3) if (later == 2) { wait_vmcnt<2 * DPS_>(); return; }
    if constexpr (DIST >= 2) if (later == 1) { wait_vmcnt<DPS_>(); return; }
    wait_vmcnt<0>();
  };
  auto wait_stage = [&](int later) { wait_stage_n(later, std::integral_constant<int, DPS>()); };
  // WO_PIPE (128 / 64-row tiles, WM = 1: their fragment sets are small): the fragments of stage
  // s+1 are read into a second register set right after the barrier that publishes stage s+1,
  // and stage s's dequant + MFMAs (first set) run while those reads are in flight; the reads no
  // longer sit between the barrier and the MFMAs of the same stage.
  constexpr bool PIPE = (WABL & WO_PIPE) != 0 && Cfg::WM == 1 && DIST >= 2;
  struct Frag {
    v8h a[2][FM];
    uint32_t rb[FN][2][2];  // B words: [j][kc][.] (4-bit: both K halves in [j][0]; 2-bit: [j][0][0])
  };
  auto read_frag = [&](int buf, Frag& f) {
    const uint8_t* As = lds + buf * SB_ + a_row;
    const uint8_t* Bs = lds + buf * SB_ + Cfg::A_BYTES + b_row;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BITS == 2) {
        f.rb[j][0][0] = *reinterpret_cast<const uint32_t*>(Bs + j * 16 * RB + g * 4);
      } else if constexpr (BITS == 4) {
        const uint2 v = *reinterpret_cast<const uint2*>(Bs + j * 16 * RB + (((g >> 1) ^ bsw) << 4) + (g & 1) * 8);
        f.rb[j][0][0] = v.x;
        f.rb[j][0][1] = v.y;
      } else {
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
          const uint2 v = *reinterpret_cast<const uint2*>(Bs + j * 16 * RB + ((g ^ bsw) << 4) + kc * 8);
          f.rb[j][kc][0] = v.x;
          f.rb[j][kc][1] = v.y;
        }
      }
    }
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const uint32_t off = (uint32_t)(((kc * 4 + g) ^ swz) << 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) f.a[kc][i] = *reinterpret_cast<const v8h*>(As + i * 2048 + off);
    }
  };
  auto dq_half = [&](const Frag& f, int kc, v8h (&b)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BITS == 2) {
        const uint32_t w = f.rb[j][0][0] >> (8 * kc);
        b[j] = wo_dequant<2>(&w, moff2, s2[j], z2[j], wok);
      } else if constexpr (BITS == 4) {
        b[j] = wo_dequant<4>(&f.rb[j][0][kc], moff2, s2[j], z2[j], wok);
      } else {
        b[j] = wo_dequant<8>(f.rb[j][kc], moff2, s2[j], z2[j], wok);
      }
    }
  };
  auto mm_half = [&](const v8h (&a)[FM], const v8h (&b)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b[j], a[i], acc[i][j], 0, 0, 0);
  };
  auto mma_frag = [&](const Frag& f) {
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      v8h b[FN];
      dq_half(f, kc, b);
      mm_half(f.a[kc], b);
    }
  };
  constexpr bool STAG = PIPE && Cfg::BM == 64 && (WABL & WO_STAG) != 0;  // (128 rows: spills)
  if constexpr (PIPE) {
   if (nst > 0) {
    load_scales(ks0 / gstages, s2, z2);
#pragma unroll
    for (int p = 0; p < DIST; ++p)
      if (p < nst) issue(p, p);
    if (DIST - 1 < nst) wait_vmcnt<(DIST - 1) * DPS>();
    else wait_stage(nst - 1);
    lds_barrier();  // stage 0 visible
    Frag fa, fb;
    read_frag(0, fa);
    int gpos = (ks0 + 1) % gstages;
    // iteration s: publish stage s+1 (wait + barrier; every wave's reads of stage s are done, so
    // the buffer of stage s-1 is free for stage s+DIST), issue it, read it into the other set,
    // then stage s's dequant + MFMAs
    auto step = [&](int s, Frag& cur, Frag& nxt) {
      if (s + 1 < nst) {
        // stages issued after s+1: min(DIST - 2, nst - 2 - s)
        if (s + DIST < nst) wait_vmcnt<(DIST - 2) * DPS>();
        else wait_stage(nst - 2 - s);
        lds_barrier();
      }
      const bool next_group = gpos == 0 && s + 1 < nst;
      gpos = gpos + 1 == gstages ? 0 : gpos + 1;
      if (next_group) load_scales((ks0 + s + 1) / gstages, s2n, z2n);
      if (s + DIST < nst) issue(s + DIST, (s + DIST) % NBUF);
      if (s + 1 < nst) read_frag((s + 1) % NBUF, nxt);
      mma_frag(cur);
      if (next_group) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          s2[j] = s2n[j];
          z2[j] = z2n[j];
        }
      }
    };
    if (!STAG || wave < 4) {
      for (int s = 0; s < nst; s += 2) {
        step(s, fa, fb);
        if (s + 1 < nst) step(s + 1, fb, fa);
      }
    } else if constexpr (STAG) {
      // late waves: stage s's second half (dequantised with stage s's scales before the barrier)
      // runs after the barrier of iteration s+1, before stage s+2's reads reuse its register set
      v8h bdef[FN];
      auto step_late = [&](int s, Frag& cur, Frag& nxt) {
        if (s + 1 < nst) {
          if (s + DIST < nst) wait_vmcnt<(DIST - 2) * DPS>();
          else wait_stage(nst - 2 - s);
          lds_barrier();
        }
        if (s > 0) mm_half(nxt.a[1], bdef);  // stage s-1, second K half
        const bool next_group = gpos == 0 && s + 1 < nst;
        gpos = gpos + 1 == gstages ? 0 : gpos + 1;
        if (next_group) load_scales((ks0 + s + 1) / gstages, s2n, z2n);
        if (s + DIST < nst) issue(s + DIST, (s + DIST) % NBUF);
        if (s + 1 < nst) read_frag((s + 1) % NBUF, nxt);
        v8h b0[FN];
        dq_half(cur, 0, b0);
        mm_half(cur.a[0], b0);
        dq_half(cur, 1, bdef);
        if (next_group) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            s2[j] = s2n[j];
            z2[j] = z2n[j];
          }
        }
      };
      for (int s = 0; s < nst; s += 2) {
        step_late(s, fa, fb);
        if (s + 1 < nst) step_late(s + 1, fb, fa);
      }
      mm_half(((nst - 1) & 1) ? fb.a[1] : fa.a[1], bdef);  // the last stage's second half
    }
    wait_vmcnt<0>();
    lds_barrier();  // ring -> epilogue staging
   }
  } else if (nst > 0 && (WABL & WO_SCLATE) != 0) {
    // A stage that opens a scale group brings the group's scale words along: one LDS-DMA piece per
    // lane (lanes 0-31: the wave's 32 columns, 2 / 4 B at lane * 4 — the DMA's LDS stride below
    // 16-B pieces) into a 1-KiB slot beside the stage's ring buffer, issued just before the stage's
    // own DMA, so the counted wait that publishes the stage covers it too: the ring never drains
    // for scales (round 3: a register load right before use, vmcnt(0) at every group boundary)
    static_assert((WABL & WO_SCLATE) == 0 || NBUF * SB_ + NBUF * 1024 <= Cfg::LDSB, "the scale slots sit past the ring");
    uint8_t* const sc_base = lds + NBUF * SB_ + wave * 128;
    load_scales(ks0 / gstages, s2, z2);
    bool one_group = false;
    if constexpr ((WABL & WO_PCH) != 0 && (WABL & WO_SPLIT) != 0 && (WABL & WO_ADEAD) == 0)
      one_group = (ks0 % gstages) + nst <= gstages;
    if constexpr ((WABL & WO_PCH) != 0 && (WABL & WO_SPLIT) != 0 && (WABL & WO_ADEAD) == 0) {
     if (one_group) {
      // WO_PCH: no scale slots, no group counters; the steady loop unrolled by NBUF (ring buffer
      // s % NBUF a constant in each copy: no per-stage offset arithmetic), the last stages with a
      // runtime buffer index
#pragma unroll
      for (int p = 0; p < DIST; ++p)
        if (p < nst) issue(p, p);
      int s = 0;
      for (; s + NBUF - 1 + DIST < nst; s += NBUF) {
        static_for<0, NBUF>([&](auto i_c) {
          constexpr int BC = decltype(i_c)::value;
          wait_vmcnt<(DIST - 1) * DPS>();
          lds_barrier();
          issue(s + BC + DIST, (BC + DIST) % NBUF);
          if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(BC);
        });
      }
      for (; s < nst; ++s) {
        if (s + DIST - 1 < nst) wait_vmcnt<(DIST - 1) * DPS>();
        else wait_stage(nst - 1 - s);
        lds_barrier();
        if (s + DIST < nst) issue(s + DIST, (s + DIST) % NBUF);
        if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(s % NBUF);
      }
     }
    }
    // WO_PCH, two stages per scale group (g128, the 64-K stages' common group size) from an even
    // stage: the loop unrolled by lcm(NBUF, 2), so each copy knows its ring buffer AND whether its
    // stage opens a group (scale slot DMA before the stage's own pieces, as below; slot read after
    // the barrier) — no group counters
    // (not for 2-bit codes: their 4-deep ring unrolled 4x spilled the 3-WG/CU build)
    constexpr bool kTwo = (WABL & WO_PCH) != 0 && (WABL & WO_SPLIT) != 0 && (WABL & WO_ADEAD) == 0 && BITS != 2;
    bool two_group = false;
    if constexpr (kTwo) two_group = !one_group && gstages == 2 && (ks0 & 1) == 0;
    if constexpr (kTwo) {
     if (two_group) {
      constexpr int L = NBUF % 2 == 0 ? NBUF : 2 * NBUF;
      const int nl = min(ncol0 + (lane & 31), N - 1);
      auto issue_sc2 = [&](int t, int buf) {  // stage t (even, > 0) opens scale group (ks0 + t) / 2
        if (lane < 32) {
          const int64_t grp = (ks0 + t) >> 1;
          if (sym) __builtin_amdgcn_global_load_lds((gbl_void_t*)(SB + grp * N + nl), (lds_void_t*)(sc_base + buf * 1024), 2, 0, 0);
          else __builtin_amdgcn_global_load_lds((gbl_void_t*)(SB + (grp * N + nl) * 2), (lds_void_t*)(sc_base + buf * 1024), 4, 0, 0);
        }
      };
      auto read_sc = [&](int buf) {
        const uint8_t* sc = sc_base + buf * 1024;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if (sym) {
            const uint32_t v = *reinterpret_cast<const uint16_t*>(sc + (j * 16 + r16) * 4);
            s2[j] = v * 0x10001u;
            z2[j] = 0;
          } else {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(sc + (j * 16 + r16) * 4);
            s2[j] = (v & 0xFFFFu) * 0x10001u;
            z2[j] = (v >> 16) * 0x10001u;
          }
        }
      };
#pragma unroll
      for (int p = 0; p < DIST; ++p)
        if (p < nst) {
          if (p > 0 && (p & 1) == 0) issue_sc2(p, p);
          issue(p, p);
        }
      int s = 0;
      for (; s + L - 1 + DIST < nst; s += L) {
        static_for<0, L>([&](auto i_c) {
          constexpr int I = decltype(i_c)::value, BC = I % NBUF, BI = (I + DIST) % NBUF;
          wait_vmcnt<(DIST - 1) * DPS>();
          lds_barrier();
          if constexpr ((I & 1) == 0) {
            if (I > 0 || s > 0) read_sc(BC);
          }
          if constexpr (((I + DIST) & 1) == 0) issue_sc2(s + I + DIST, BI);
          issue(s + I + DIST, BI);
          if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(BC);
        });
      }
      for (; s < nst; ++s) {
        if (s + DIST - 1 < nst) wait_vmcnt<(DIST - 1) * DPS>();
        else wait_stage(nst - 1 - s);
        lds_barrier();
        if (s > 0 && (s & 1) == 0) read_sc(s % NBUF);
        if (s + DIST < nst) {
          if (((s + DIST) & 1) == 0) issue_sc2(s + DIST, (s + DIST) % NBUF);
          issue(s + DIST, (s + DIST) % NBUF);
        }
        if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(s % NBUF);
      }
     }
    }
    if (!one_group && !two_group) {
    const int nl = min(ncol0 + (lane & 31), N - 1);
    int ipos = ks0 % gstages, igrp = ks0 / gstages;  // issue stream: stage t's place in its group
    int cpos = ipos;                                   // compute stream
    auto issue_sc = [&](int t, int buf) {
      if (t > 0 && ipos == 0 && lane < 32) {
        if (sym) __builtin_amdgcn_global_load_lds((gbl_void_t*)(SB + (int64_t)igrp * N + nl), (lds_void_t*)(sc_base + buf * 1024), 2, 0, 0);
        else __builtin_amdgcn_global_load_lds((gbl_void_t*)(SB + ((int64_t)igrp * N + nl) * 2), (lds_void_t*)(sc_base + buf * 1024), 4, 0, 0);
      }
      if (++ipos == gstages) {
        ipos = 0;
        ++igrp;
      }
    };
#pragma unroll
    for (int p = 0; p < DIST; ++p)
      if (p < nst) {
        issue_sc(p, p);
        issue(p, p);
      }
    int bc = 0, bi = DIST % NBUF;  // s % NBUF, (s + DIST) % NBUF
    // STEADY: stage s + DIST exists (one constant wait, an unconditional issue); the tail waits by
    // the count of stages still in flight (WO_SPLIT: two loops; else one loop with both tests)
    auto step = [&](int s, auto steady_c) {
      constexpr bool STEADY = decltype(steady_c)::value;
      if constexpr ((WABL & WO_SPLIT) != 0 && (WABL & WO_ADEAD) != 0) {
        if (a_live) {
          if constexpr (STEADY) wait_vmcnt<(DIST - 1) * DPS>();
          else wait_stage(nst - 1 - s);
        } else {
          if constexpr (STEADY) wait_vmcnt<(DIST - 1) * (DPS - GA)>();
          else wait_stage_n(nst - 1 - s, std::integral_constant<int, DPS - GA>());
        }
      } else if constexpr ((WABL & WO_SPLIT) != 0) {
        if constexpr (STEADY) wait_vmcnt<(DIST - 1) * DPS>();
        else wait_stage(nst - 1 - s);
      } else {
        if (s + DIST - 1 < nst) wait_vmcnt<(DIST - 1) * DPS>();
        else wait_stage(nst - 1 - s);
      }
      lds_barrier();
      if (s > 0 && cpos == 0) {  // stage s opens a group: its scales sit in the slot of its buffer
        const uint8_t* sc = sc_base + bc * 1024;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if (sym) {
            const uint32_t v = *reinterpret_cast<const uint16_t*>(sc + (j * 16 + r16) * 4);
            s2[j] = v * 0x10001u;
            z2[j] = 0;
          } else {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(sc + (j * 16 + r16) * 4);
            s2[j] = (v & 0xFFFFu) * 0x10001u;
            z2[j] = (v >> 16) * 0x10001u;
          }
        }
      }
      if (++cpos == gstages) cpos = 0;
      if constexpr ((WABL & WO_SPLIT) != 0) {
        if constexpr (STEADY) {
          issue_sc(s + DIST, bi);
          issue(s + DIST, bi);
        }
      } else {
        if (s + DIST < nst) {
          issue_sc(s + DIST, bi);
          issue(s + DIST, bi);
        }
      }
      if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(bc);
      bc = bc + 1 == NBUF ? 0 : bc + 1;
      bi = bi + 1 == NBUF ? 0 : bi + 1;
    };
    if constexpr ((WABL & WO_SPLIT) != 0) {
      int s = 0;
      for (; s + DIST < nst; ++s) step(s, std::true_type());
      for (; s < nst; ++s) step(s, std::false_type());
    } else {
      for (int s = 0; s < nst; ++s) step(s, std::true_type());
    }
    }  // (!one_group)
    wait_vmcnt<0>();
    lds_barrier();  // ring -> epilogue staging
  } else if (nst > 0) {
    load_scales(ks0 / gstages, s2, z2);
#pragma unroll
    for (int p = 0; p < DIST; ++p)
      if (p < nst) issue(p, p);
    int gpos = (ks0 + 1) % gstages;  // (ks0 + s + 1) % gstages, kept as a counter (no divide per stage)
    for (int s = 0; s < nst; ++s) {
      // stages s+1 .. min(s+DIST-1, nst-1) were issued after s (younger scale loads only make the
      // in-order count wait longer, never shorter); the steady state is one constant wait
      if (s + DIST - 1 < nst) wait_vmcnt<(DIST - 1) * DPS>();
      else wait_stage(nst - 1 - s);
      lds_barrier();  // stage s visible to every wave; buffer (s-1) % NBUF released by all
      // next group's scales BEFORE this iteration's DMA: the wait the compiler places before their
      // use then leaves the (younger) DMA in flight instead of draining it
      const bool next_group = gpos == 0 && s + 1 < nst;
      gpos = gpos + 1 == gstages ? 0 : gpos + 1;
      if (next_group) load_scales((ks0 + s + 1) / gstages, s2n, z2n);  // lands under this stage's MFMAs
      if (s + DIST < nst) issue(s + DIST, (s + DIST) % NBUF);
      if constexpr ((WABL & ABL_WO_NOCOMPUTE) == 0) compute(s % NBUF);
      if (next_group) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          s2[j] = s2n[j];
          z2[j] = z2n[j];
        }
      }
    }
    wait_vmcnt<0>();
    lds_barrier();  // ring -> epilogue staging
  }
  if (!splitk_reduce<Cfg::NT>(acc, sk, lds)) return;  // split-K: only the last slice writes C
  epilogue_v3<Cfg, QT_F16, (WABL & WO_SILU) != 0>(mt, acc, nullptr, nullptr, C, m0, n0, lds);
}

template <int ABL, int QM>  // QM: quant types compiled in (bit 1 << QType), as gg_v3_kernel
__global__ __launch_bounds__(512, 2) void gg_v2_kernel(GGArgs args) {
  // + the int paths' scale stash: SA at [LDS_BYTES, +2*BM), SB at [LDS_BYTES + 512, +512)
  __shared__ __attribute__((aligned(16))) uint8_t lds[(ABL & V2_B3) ? 160 * 1024 : V2Cfg<256>::LDS_BYTES + V2_LDS_EXTRA];
  if constexpr ((ABL & V2_TRACE) != 0) trace_mark(0);
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const GGMeta mt = args.meta[td.prob];
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[td.prob]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[td.prob]);
  const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
  const _Float16* SB = static_cast<const _Float16*>(args.ptr_SB[td.prob]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[td.prob]);
  // 0: 256 rows, 1: 128, 2: 64 (fp16 / weight-only only: the int bodies sit at the 256-VGPR edge
  // and a third inlined height made the compiler spill inside their K loops)
  const int cls = td.cls & 0xFF;
  SplitK sk;
  sk.ks0 = td.ks0;
  sk.nst = td.ks1 - td.ks0;
  sk.idx = (td.cls >> 8) & 0xFF;
  sk.nsplit = (td.cls >> 16) & 0xFF;
  sk.slab = td.slab;
  sk.grp = td.grp;
  sk.slabs = args.slabs;
  sk.counters = args.counters;
  if ((QM & (1 << QT_I8)) && mt.qtype == QT_I8) {
    if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_I8, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v2<V2Cfg<128>, QT_I8, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);  // no 64-row class
  } else if constexpr ((ABL & kAblMask) != 0) {
    return;  // ablation builds time the int8 path only
  } else if ((QM & (1 << QT_I4)) && mt.qtype == QT_I4) {
    if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_I4, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v2<V2Cfg<128>, QT_I4, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);  // no 64-row class
  } else if ((QM & (1 << QT_I4G)) && mt.qtype == QT_I4G) {
    if (cls == 0) gg_tile_g128<V2Cfg<256>>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
    else gg_tile_g128<V2Cfg<128>>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
  } else if ((QM & (1 << QT_F8)) && mt.qtype == QT_F8) {
    // one K = 128 MFMA per stage: no K halves to stagger, so the plain v2 mainloop (two 64-KiB
    // stages, inside either LDS image)
    constexpr int F8ABL = ABL & ~(V2_STAGGER | V2_B3);
    if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_F8, F8ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v2<V2Cfg<128>, QT_F8, F8ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);  // no 64-row class
  } else if ((QM & (1 << QT_BF16)) && mt.qtype == QT_BF16) {
    if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_BF16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_v2<V2Cfg<128>, QT_BF16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v2<V2Cfg<64>, QT_BF16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_F16)) && mt.qtype == QT_F16) {
    if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_F16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_v2<V2Cfg<128>, QT_F16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v2<V2Cfg<64>, QT_F16, ABL>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_W4A16)) && mt.qtype == QT_W4A16) {
    constexpr int WABL = ABL & (kWoAblMask | WO_PIPE | WO_STAG);
    if (cls == 0) gg_tile_wo<WoCfg<256>, 4, WABL>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 4, WABL>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_wo<WoCfg<64, 1>, 4, WABL>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_W8A16)) && mt.qtype == QT_W8A16) {
    constexpr int WP = ABL & (WO_PIPE | WO_STAG);
    if (cls == 0) gg_tile_wo<WoCfg<256>, 8, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 8, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_wo<WoCfg<64, 1>, 8, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_W2A16)) && mt.qtype == QT_W2A16) {
    constexpr int WP = ABL & (WO_PIPE | WO_STAG);
    if (cls == 0) gg_tile_wo<WoCfg<256>, 2, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 2, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_wo<WoCfg<64, 1>, 2, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  }
  if constexpr ((ABL & V2_TRACE) != 0) {
    if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks) {
      wait_vmcnt<0>();
      uint64_t hw = ((uint64_t)(__builtin_amdgcn_s_getreg((19 << 11) | 20) & 0xF) << 32) |  // XCC_ID
                    ((uint64_t)(mt.qtype & 0xF) << 36) | ((uint64_t)(cls & 0xFF) << 40) |
                    ((uint64_t)(sk.nst & 0xFFFF) << 48) | (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
      g_gg_trace[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
      g_gg_trace[blockIdx.x * 4 + 3] = hw;
    }
  }
}


// ============================================================================================
// wo2: the 64-row weight-only tile (gg_tile_wo, 1 x 8 waves, 64 x 32 wave tiles) in a kernel small
// enough for TWO workgroups per CU: <= 128 VGPRs (4 waves per SIMD) and a 78-KiB LDS image (ring
// of 4 stages for 4-bit codes, 3 for 8-bit, 6 for 2-bit; the 32-KiB epilogue staging). For small
// batches (routed experts of ~35 rows) the 64-row tile is bound by its per-stage instruction
// stream and barrier latency, not by the weight stream: a second resident workgroup fills the
// other one's waits. Planned with 64-row tiles only (variant geometry bm = 64, no tail classes).
// ============================================================================================
// NWG = 3: three workgroups per CU (<= 80 VGPRs, 52-KiB image: 3 / 2 / 4 stages)
template <int NWG>
constexpr int wo2_lds_bytes() { return NWG == 3 ? 52 * 1024 : 78 * 1024; }
template <int ABL, int QM, int NWG = 2>
__global__ __launch_bounds__(512, 2 * NWG) void gg_wo2_kernel(GGArgs args) {
  constexpr int WO2_LDS_BYTES = wo2_lds_bytes<NWG>();
  __shared__ __attribute__((aligned(16))) uint8_t lds[WO2_LDS_BYTES];
  if constexpr ((ABL & V2_TRACE) != 0) trace_mark(0);
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const GGMeta mt = args.meta[td.prob];
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[td.prob]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[td.prob]);
  const _Float16* SB = static_cast<const _Float16*>(args.ptr_SB[td.prob]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[td.prob]);
  SplitK sk;
  sk.ks0 = td.ks0;
  sk.nst = td.ks1 - td.ks0;
  sk.idx = (td.cls >> 8) & 0xFF;
  sk.nsplit = (td.cls >> 16) & 0xFF;
  sk.slab = td.slab;
  sk.grp = td.grp;
  sk.slabs = args.slabs;
  sk.counters = args.counters;
  typedef WoCfg<64, 1, WO2_LDS_BYTES> Cfg;
  constexpr int WP = ABL & (WO_PIPE | WO_STAG | WO_SCLATE | WO_ANDOR | WO_MSKIP | WO_SPLIT | WO_NIBPOS | WO_ADEAD | WO_BUF | WO_SILU | WO_PCH | kWoAblMask);  // (not V2_TRACE)  // (ablations: lab builds only)
  if ((QM & (1 << QT_I8)) && mt.qtype == QT_I8) {
    // w8a8 beside the weight-only problems (the reference's small-batch w4a16 + w8a8 pairing,
    // hz_fused.cuh:14-125): the plain v2 int8 body on a 64 x 128 tile, 4 x 2 waves of 16 x 64
    // (two 24-KiB stages + the scale stash: 49 KiB)
    const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
    gg_tile_v2<V2Cfg<64, 128, 4, 2>, QT_I8, 0>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_F16)) && mt.qtype == QT_F16) {
    // fp16 on the same 64 x 128 tile (two 24-KiB stages of 64 K)
    gg_tile_v2<V2Cfg<64, 128, 4, 2>, QT_F16, 0>(mt, A, B, nullptr, nullptr, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_I4)) && mt.qtype == QT_I4) {
    // w4a4 on the same 64 x 128 tile (two 24-KiB stages of 256 K, nibbles widened to int8 MFMA)
    const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
    gg_tile_v2<V2Cfg<64, 128, 4, 2>, QT_I4, 0>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_W4A16)) && mt.qtype == QT_W4A16) gg_tile_wo<Cfg, 4, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  else if ((QM & (1 << QT_W8A16)) && mt.qtype == QT_W8A16) gg_tile_wo<Cfg, 8, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  else if ((QM & (1 << QT_W2A16)) && mt.qtype == QT_W2A16) gg_tile_wo<Cfg, 2, WP>(mt, A, B, SB, C, td.m0, td.n0, lds, sk);
  if constexpr ((ABL & V2_TRACE) != 0) {  // (as gg_v2_kernel; the class field holds the problem index)
    if (threadIdx.x == 0 && blockIdx.x < kTraceBlocks) {
      wait_vmcnt<0>();
      uint64_t hw = ((uint64_t)(__builtin_amdgcn_s_getreg((19 << 11) | 20) & 0xF) << 32) |
                    ((uint64_t)(mt.qtype & 0xF) << 36) | ((uint64_t)(td.prob & 0xFF) << 40) |
                    ((uint64_t)(sk.nst & 0xFFFF) << 48) | (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_gg_trace[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
      g_gg_trace[blockIdx.x * 4 + 3] = hw;
    }
  }
}

// ============================================================================================
// v2p: the persistent v2x. One 512-thread workgroup per CU walks a planned list of tiles
// (TileDesc table laid out [k][workgroup], k-th tile of workgroup w at k * gridDim.x + w; the list
// ends at the first prob < 0). The tile body is v2x's mainloop (3-stage B ring, buffer-form LDS-DMA
// spread over the MFMAs, early waves issuing their partners' pieces) with two hand-offs between
// consecutive tiles of a workgroup instead of a kernel-level block boundary:
//   * after tile i's last barrier every ring slot is free: tile i+1's stage 0 (A and B) and B(1)
//     are issued into A slot 0 / B slots 0-1 BEFORE tile i's epilogue (same quant type and tile
//     height only), so their latency hides under the epilogue;
//   * tile i's epilogue stages C through LDS in the slots that prefetch does not touch (A slot 1
//     for waves 0-3, B slot 2 for waves 4-7, 64 rows per pass) and issues exactly WTM / 8 buffer
//     stores per wave (masked lanes get an out-of-range offset instead of a branch), so tile i+1's
//     first wait can count them: vmcnt(stores + B(1) pieces) leaves the stores draining under the
//     next tile's first MFMAs.
// LDS map: A slots [0, 32K) [32K, 64K); B ring [64K, 96K) [96K, 128K) [128K, 160K).
// ============================================================================================
constexpr int P_ASLOT = 32768, P_BBASE = 65536, P_BSLOT = 32768;

struct PTile {  // one planned tile with its problem resolved
  GGMeta mt;
  const uint8_t* A;
  const uint8_t* B;
  const _Float16* SA;
  const _Float16* SB;
  _Float16* C;
  int m0, n0, cls;
  SplitK sk;
};

// Resolve tile slot `idx` of the table (false: an empty slot). `a` is passed through an opaque
// copy by the caller where a second resolve must really reload (so the compiler does not keep the
// first resolve's ~40 scalar registers live across a mainloop instead).
// Wave-uniform copies (v_readfirstlane): once the persistent kernel has stored C, hipcc can no
// longer prove the plan tables unmodified and loads them with vector loads; without these the buffer
// resources built from them land in VGPRs and every LDS-DMA becomes a waterfall loop
// (cdna_hip_programming.md T20).
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uni(int64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <class T>
__device__ __forceinline__ T* uni(T* p) {
  return reinterpret_cast<T*>(uni((int64_t)reinterpret_cast<uintptr_t>(p)));
}

// Scalar (SMEM) loads of the plan tables, by inline asm: hipcc turns these loads into VECTOR loads
// once the persistent kernel has stored C (it cannot prove the tables unclobbered), and a vector load
// waits behind every older store and LDS-DMA (in-order vmcnt) — 1.5-2 us per tile boundary. SMEM
// loads count on lgkmcnt instead. The tables are read-only during a launch (written by the host).
typedef int32_t v8s_t __attribute__((ext_vector_type(8)));
typedef int32_t v16s_t __attribute__((ext_vector_type(16)));
// (each asm statement waits for its own loads: a register an asm statement defines may be read by
// the compiler right after it, so no load may be left in flight across statements; the outputs are
// early-clobber because several loads share one statement)
__device__ __forceinline__ TileDesc p_tile(const GGArgs& a, int idx) {
  v8s_t v;
  asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(v) : "s"(a.tiles + idx) : "memory");
  return __builtin_bit_cast(TileDesc, v);
}
// problem row `prob`: its GGMeta and its five pointers, one batch of scalar loads
__device__ __forceinline__ void p_problem(const GGArgs& a, int prob, v16s_t& meta, uint64_t& pa, uint64_t& pb,
                                          uint64_t& psa, uint64_t& psb, uint64_t& pc) {
  asm volatile(
      "s_load_dwordx16 %0, %6, 0x0\n\t"
      "s_load_dwordx2 %1, %7, 0x0\n\t"
      "s_load_dwordx2 %2, %8, 0x0\n\t"
      "s_load_dwordx2 %3, %9, 0x0\n\t"
      "s_load_dwordx2 %4, %10, 0x0\n\t"
      "s_load_dwordx2 %5, %11, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(meta), "=&s"(pa), "=&s"(pb), "=&s"(psa), "=&s"(psb), "=&s"(pc)
      : "s"(a.meta + prob), "s"(a.ptr_A + prob), "s"(a.ptr_B + prob), "s"(a.ptr_SA + prob), "s"(a.ptr_SB + prob),
        "s"(a.ptr_C + prob)
      : "memory");
}
__device__ __forceinline__ int p_qtype(const GGArgs& a, int prob) {
  int q;
  asm volatile("s_load_dword %0, %1, 0xc\n\ts_waitcnt lgkmcnt(0)" : "=&s"(q) : "s"(a.meta + prob) : "memory");
  return q;
}

__device__ __forceinline__ bool p_resolve(const GGArgs& a, int idx, PTile& pt) {
  const TileDesc td = p_tile(a, idx);
  const int prob = uni(td.prob);
  if (prob < 0) return false;
  v16s_t mv;
  uint64_t pa, pb, psa, psb, pc;
  p_problem(a, prob, mv, pa, pb, psa, psb, pc);
  const GGMeta m = __builtin_bit_cast(GGMeta, mv);
  pt.mt.M = uni(m.M);
  pt.mt.N = uni(m.N);
  pt.mt.K = uni(m.K);
  pt.mt.qtype = uni(m.qtype);
  pt.mt.tiles_n = uni(m.tiles_n);
  pt.mt.tile_begin = uni(m.tile_begin);
  pt.mt.kbytes = uni(m.kbytes);
  pt.mt.reserved = uni(m.reserved);
  pt.mt.lda_b = uni(m.lda_b);
  pt.mt.ldb_b = uni(m.ldb_b);
  pt.mt.ldc = uni(m.ldc);
  pt.mt.reserved2 = uni(m.reserved2);
  pt.A = reinterpret_cast<const uint8_t*>(pa);
  pt.B = reinterpret_cast<const uint8_t*>(pb);
  pt.SA = reinterpret_cast<const _Float16*>(psa);
  pt.SB = reinterpret_cast<const _Float16*>(psb);
  pt.C = reinterpret_cast<_Float16*>(pc);
  pt.m0 = uni(td.m0);
  pt.n0 = uni(td.n0);
  const int cls = uni(td.cls);
  pt.cls = cls & 0xFF;
  pt.sk.ks0 = uni(td.ks0);
  pt.sk.nst = uni(td.ks1) - pt.sk.ks0;
  pt.sk.idx = (cls >> 8) & 0xFF;
  pt.sk.nsplit = (cls >> 16) & 0xFF;
  pt.sk.slab = uni(td.slab);
  pt.sk.grp = uni(td.grp);
  pt.sk.slabs = a.slabs;
  pt.sk.counters = a.counters;
  return true;
}

__device__ __forceinline__ GGArgs p_opaque(const GGArgs& a) {
  GGArgs o = a;
  asm volatile("" : "+s"(o.tiles), "+s"(o.meta), "+s"(o.ptr_A), "+s"(o.ptr_B));
  asm volatile("" : "+s"(o.ptr_SA), "+s"(o.ptr_SB), "+s"(o.ptr_C));
  return o;
}

struct PTileResult {
  bool pref;   // the next tile's first stages were issued
  int stores;  // buffer stores this wave issued in the epilogue (all after the prefetch)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt_rt(int n) {  // runtime count, bounded by N (unrolled compare chain)
  if constexpr (N > 0) {
    if (n >= N) {
      wait_vmcnt<N>();
      return;
    }
    wait_vmcnt_rt<N - 1>(n);
  } else {
    wait_vmcnt<0>();
  }
}

template <class Cfg, int QT, int TRACE = 0>
__device__ __forceinline__ PTileResult gg_tile_v2p(const GGArgs& args, int cur_idx, int nx_idx, bool prefetched,
                                                   int s_prev, uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB;
  typedef typename AccT<QT>::type acc_t;
  typedef V2Half<Cfg, QT, 0> Half;
  constexpr bool EDMA = QT != QT_I4;  // int4 half stages carry twice the MFMAs: no slack in the early waves
  constexpr int HALFW = Cfg::WM * Cfg::WN / 2;
  constexpr int NH = Half::kMfma, NR = Half::kReads, ND = GA + GB;
  constexpr int NDE = EDMA ? 2 * ND : ND;
  constexpr int KSE = 4 * NDE <= NH ? 4 : (NH / NDE > 0 ? NH / NDE : 1);
  constexpr int RESTE = NH - KSE * NDE > 0 ? NH - KSE * NDE : 0;
  constexpr int SPW = Cfg::WTM / 8;  // epilogue buffer stores per wave
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // per tile: nothing lane-derived is hoisted out of the persistent loop
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const bool early = wave < HALFW;
  const int pw = EDMA ? (early ? 2 : 0) : 1;  // LDS-DMA pieces this wave issues per (operand, row group)
  PTile t;
  p_resolve(args, cur_idx, t);
  const GGMeta& mt = t.mt;
  const int kbytes = mt.kbytes;
  const int nst = t.sk.nst, ks0 = t.sk.ks0;
  const int M = mt.M, N = mt.N;

  auto abuf = [&](int s) { return lds + (s & 1) * P_ASLOT; };
  auto bbuf = [&](int s) { return lds + P_BBASE + (s % 3) * P_BSLOT; };
  // buffer resources of a tile (rows past M / N read as zeros) and its fixed lane offsets
  auto rsrc = [&](const uint8_t* base, int64_t ld, int rows) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)(rows * ld), 0x00020000);
  };
  auto lane_off = [&](int G, int j, int64_t ld) {
    const int row = (wave * G + j) * 8 + (lane >> 3);
    return (uint32_t)(row * ld) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
  };
  // the pieces of one operand of stage kb (bytes) into dst: this wave's rows, and (EDMA, early
  // waves) its partner's rows (8 * G * HALFW further, the same swizzle)
  auto dma = [&](const __amdgpu_buffer_rsrc_t& rs, const uint32_t* vo, int G, int64_t ld, int kb, int kbytes_,
                 bool full, uint8_t* dst) {
    if (EDMA && !early) return;
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int w2 = 0; w2 < (EDMA ? 2 : 1); ++w2) {
      const int ww = wave + w2 * HALFW;
      const uint32_t radd = (uint32_t)(w2 * 8 * G * HALFW * ld);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= G) break;
        const int kc = (p ^ ((((wave * G + j) * 8 + rsub) >> 1) & 7)) << 4;
        const bool in = full || kb + kc < kbytes_;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + (ww * G + j) * 1024), 16,
                                                 in ? vo[j] + radd : 0x80000000u, kb, 0, 0);
      }
    }
  };

  const __amdgpu_buffer_rsrc_t rsA = rsrc(t.A + (int64_t)t.m0 * mt.lda_b, mt.lda_b, min(M - t.m0, Cfg::BM));
  const __amdgpu_buffer_rsrc_t rsB = rsrc(t.B + (int64_t)t.n0 * mt.ldb_b, mt.ldb_b, min(N - t.n0, Cfg::BN));
  uint32_t voA[4], voB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    voA[j] = j < GA ? lane_off(GA, j, mt.lda_b) : 0u;
    voB[j] = j < GB ? lane_off(GB, j, mt.ldb_b) : 0u;
  }
  const int nst_full = (ks0 + nst) * Cfg::BKB > kbytes ? nst - 1 : nst;
  auto full_stage = [&](int s) { return s < nst_full; };
  auto dma_a = [&](int s, bool full) { dma(rsA, voA, GA, mt.lda_b, (ks0 + s) * Cfg::BKB, kbytes, full, abuf(s)); };
  auto dma_b = [&](int s, bool full) { dma(rsB, voB, GB, mt.ldb_b, (ks0 + s) * Cfg::BKB, kbytes, full, bbuf(s)); };
  auto dma_steady = [&](int s) {
    dma_a(s + 1, true);
    dma_b(s + 2, true);
  };
  auto dma_generic = [&](int s) {
    if (s + 1 < nst) dma_a(s + 1, full_stage(s + 1));
    if (s + 2 < nst) dma_b(s + 2, full_stage(s + 2));
  };
  const int nsteady = nst_full - 2;
  auto stage_wait = [&](int s) {
    if (s + 2 < nst) wait_vmcnt<(EDMA ? 2 : 1) * GB>();
    else wait_vmcnt<0>();
  };
  const int swz = (r16 >> 1) & 7;
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u;
  const uint32_t b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  auto hread = [&](Half& f, int s, int h) { f.read(abuf(s), bbuf(s), a_row, b_row, swz, g, h); };
  acc_t acc[FM][FN];
  auto hmma = [&](const Half& f) { f.mma(acc); };
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  // (TRACE, lab diagnostics: per tile slot {start, mainloop end, epilogue issued, info} in g_gg_trace)
  [[maybe_unused]] auto tmark = [&](int slot) {
    if constexpr (TRACE != 0) {
      if (tid == 0 && cur_idx < kTraceBlocks) g_gg_trace[cur_idx * 4 + slot] = __builtin_amdgcn_s_memrealtime();
    }
  };
  tmark(0);
  // ---- prologue: stage 0 + B(1) (issued by the previous tile when prefetched) ----
  if (nst > 0) {
    if (!prefetched) {
      dma_a(0, full_stage(0));
      dma_b(0, full_stage(0));
      if (nst > 1) dma_b(1, full_stage(1));
      stage_wait(-1);
    } else {
      // outstanding, oldest first: [A(0), B(0), B(1)] (prefetch) then the previous epilogue's
      // s_prev stores; A(0) and B(0) must have landed
      wait_vmcnt_rt<3 * 16>(s_prev + (nst > 1 ? pw * GB : 0));
    }
    lds_barrier();
    Half fr;
    if (!early) {  // late waves
      dma_generic(0);
      hread(fr, 0, 0);
      hmma(fr);
      hread(fr, 0, 1);
      stage_wait(0);
      lds_barrier();
      int s = 1;
      for (; s < nsteady; ++s) {
        dma_steady(s);
        hmma(fr);
        hread(fr, s, 0);
        hmma(fr);
        hread(fr, s, 1);
        if constexpr (EDMA) {
          __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        } else {
#pragma unroll
          for (int q = 0; q < ND; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, KSE, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, RESTE, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        }
        stage_wait(s);
        lds_barrier();
      }
      for (; s < nst; ++s) {
        dma_generic(s);
        hmma(fr);
        hread(fr, s, 0);
        hmma(fr);
        hread(fr, s, 1);
        stage_wait(s);
        lds_barrier();
      }
      hmma(fr);
    } else {  // early waves
      int s = 0;
      for (; s < nsteady; ++s) {
        hread(fr, s, 0);
        dma_steady(s);
        hmma(fr);
        hread(fr, s, 1);
        hmma(fr);
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
        for (int q = 0; q < NDE; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, KSE, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, RESTE, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NH, 0);
        stage_wait(s);
        lds_barrier();
      }
      for (; s < nst; ++s) {
        dma_generic(s);
        hread(fr, s, 0);
        hmma(fr);
        hread(fr, s, 1);
        hmma(fr);
        stage_wait(s);
        lds_barrier();
      }
    }
  } else {
    __syncthreads();
  }

  tmark(1);
  // ---- between the tiles: scales (int paths) into registers, then the next tile's first stages ----
  // (both tiles re-resolved from memory: nothing of the mainloop's setup stays live across it)
  int ci = __builtin_amdgcn_readfirstlane(cur_idx), ni = __builtin_amdgcn_readfirstlane(nx_idx);
  asm volatile("" : "+s"(ci), "+s"(ni));  // opaque indices: the resolves below reload (scalar loads)
  PTile nx;
  p_resolve(args, ci, t);
  const bool nx_ok = ni >= 0 && p_resolve(args, ni, nx) && nx.mt.qtype == QT && nx.cls == t.cls;
  int etid = tid;
  asm volatile("" : "+v"(etid));  // keep the lane decomposition out of the mainloop's live set
  const int e_lane = etid & 63, e_r16 = e_lane & 15, e_g = e_lane >> 4;
  const int mrow0 = t.m0 + wm * Cfg::WTM, ncol0 = t.n0 + wn * Cfg::WTN;
  const int Me = t.mt.M, Ne = t.mt.N;
  [[maybe_unused]] _Float16 sai[FM];
  [[maybe_unused]] uint2 sbw[FN];
  if constexpr (qt_scaled(QT)) {  // (global, not flat, loads: a flat load would make hipcc wait vmcnt(0))
    typedef const __attribute__((address_space(1))) _Float16 gh_t;
    typedef const __attribute__((address_space(1))) uint64_t gu64_t;
    gh_t* sa = (gh_t*)(t.SA);
    gh_t* sb = (gh_t*)(t.SB);
#pragma unroll
    for (int i = 0; i < FM; ++i) sai[i] = sa[min(mrow0 + i * 16 + e_r16, Me - 1)];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = min(ncol0 + j * 16 + 4 * e_g, Ne - 4);  // N % 8 == 0: a 4-column group stays in range
      sbw[j] = __builtin_bit_cast(uint2, *(gu64_t*)(sb + c));
    }
  }
  const bool narrow = (int64_t)Cfg::WTM * t.mt.ldc < (int64_t)1 << 29;  // C byte offsets < 2^30
  const bool split = t.sk.nsplit > 1;
#ifdef V2P_NO_PREF
  const bool pref = false && nx_ok;
#else
  const bool pref = nx_ok && narrow && !split && nst > 0;
#endif
  int npref = 0;
  if (pref) {
    const GGMeta& nm = nx.mt;
    const __amdgpu_buffer_rsrc_t nA = rsrc(nx.A + (int64_t)nx.m0 * nm.lda_b, nm.lda_b, min(nm.M - nx.m0, Cfg::BM));
    const __amdgpu_buffer_rsrc_t nB = rsrc(nx.B + (int64_t)nx.n0 * nm.ldb_b, nm.ldb_b, min(nm.N - nx.n0, Cfg::BN));
    uint32_t vA[4], vB[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      vA[j] = j < GA ? lane_off(GA, j, nm.lda_b) : 0u;
      vB[j] = j < GB ? lane_off(GB, j, nm.ldb_b) : 0u;
    }
    const int nks0 = nx.sk.ks0, nnst = nx.sk.nst;
    const int nfull = (nks0 + nnst) * Cfg::BKB > nm.kbytes ? nnst - 1 : nnst;
    if (nnst > 0) {
      dma(nA, vA, GA, nm.lda_b, nks0 * Cfg::BKB, nm.kbytes, 0 < nfull, abuf(0));
      dma(nB, vB, GB, nm.ldb_b, nks0 * Cfg::BKB, nm.kbytes, 0 < nfull, bbuf(0));
      npref = pw * (GA + GB);
      if (nnst > 1) {
        dma(nB, vB, GB, nm.ldb_b, (nks0 + 1) * Cfg::BKB, nm.kbytes, 1 < nfull, bbuf(1));
        npref += pw * GB;
      }
    }
  }
  if constexpr (qt_scaled(QT)) wait_vmcnt_rt<3 * 16>(npref);  // the scale loads (older than the prefetch)
  if (split && !splitk_reduce<Cfg::NT>(acc, t.sk, lds)) return PTileResult{false, 0};

  // ---- epilogue: per-wave staging in the slots the prefetch leaves alone, 64 rows per pass ----
  constexpr int RP = Cfg::WTM < 64 ? Cfg::WTM : 64;
  uint8_t* reg = early ? lds + P_ASLOT + wave * 8192 : lds + P_BBASE + 2 * P_BSLOT + (wave - HALFW) * 8192;
  const int64_t ldc = t.mt.ldc;
  _Float16* const cbase = t.C + (int64_t)mrow0 * ldc + ncol0;  // wave-uniform
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(cbase, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int pass = 0; pass < Cfg::WTM / RP; ++pass) {
#pragma unroll
    for (int i = pass * RP / 16; i < (pass + 1) * RP / 16; ++i) {
      const int ml = i * 16 + e_r16 - pass * RP;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        uint2 pk;
        if constexpr (QT == QT_F16 || QT == QT_BF16) pk = pack4_f16(acc[i][j]);
        else pk = scale_pack4<(QT == QT_I4) ? 8 : 0>(acc[i][j], sai[i], sbw[j]);
        const int q = 2 * j + (e_g >> 1);
        *reinterpret_cast<uint2*>(reg + ml * 128 + ((q ^ (ml & 7)) << 4) + (e_g & 1) * 8) = pk;
      }
    }
    // (a wave reads back only its own region: LDS keeps one wave's accesses in order)
#pragma unroll
    for (int it = 0; it < RP / 8; ++it) {
      const int rl = it * 8 + (e_lane >> 3), q = e_lane & 7;
      const uint4 v = *reinterpret_cast<const uint4*>(reg + rl * 128 + ((q ^ (rl & 7)) << 4));
      const int row = pass * RP + rl;
      const int m = mrow0 + row, n = ncol0 + q * 8;
      if (narrow) {
        typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
        const v4u_ d = {v.x, v.y, v.z, v.w};
        const uint32_t off = (m < Me && n < Ne) ? (uint32_t)(((int64_t)row * ldc + q * 8) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(d, rsC, (int)off, 0, 16 /* sc1 */);
      } else if (m < Me && n < Ne) {
        *reinterpret_cast<uint4*>(cbase + (int64_t)row * ldc + q * 8) = v;
      }
    }
  }
  if constexpr (TRACE != 0) {
    if (tid == 0 && cur_idx < kTraceBlocks) {
      g_gg_trace[cur_idx * 4 + 2] = __builtin_amdgcn_s_memrealtime();
      g_gg_trace[cur_idx * 4 + 3] = ((uint64_t)(__builtin_amdgcn_s_getreg((19 << 11) | 20) & 0xF) << 32) |
                                    ((uint64_t)(QT & 0xF) << 36) | ((uint64_t)(t.cls & 0xFF) << 40) |
                                    ((uint64_t)(nst & 0xFFFF) << 48) | (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
  }
  return PTileResult{pref, pref ? SPW : 0};
}

template <int QM, int TRACE = 0>
__global__ __launch_bounds__(512, 2) void gg_v2p_kernel(GGArgs args) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
  const int G = gridDim.x;
  auto family = [](int qt) { return qt == QT_F16 || qt == QT_I8 || qt == QT_I4 || qt == QT_BF16; };
  bool pref = false;
  int s_prev = 0;
  for (int k = 0;; ++k) {
    const int idx = k * G + blockIdx.x;
    const TileDesc td = p_tile(args, idx);
    const int prob = uni(td.prob);
    if (prob < 0) break;
    const int nx_idx = uni(p_tile(args, idx + G).prob) >= 0 ? idx + G : -1;
    const int qt = uni(p_qtype(args, prob)), cls = uni(td.cls) & 0xFF;
    if (!pref && k > 0) __syncthreads();  // the previous tile's LDS use is over for every wave
    PTileResult r{false, 0};
    bool done = false;
#define MXMOE_V2P(Q, BMC)                                                                              \
  if (!done && (QM & (1 << Q)) && qt == Q && cls == BMC) {                                             \
    r = gg_tile_v2p<V2Cfg<(BMC) == 0 ? 256 : (BMC) == 1 ? 128 : 64>, Q, TRACE>(args, idx, nx_idx, pref, s_prev, lds); \
    done = true;                                                                                       \
  }
    MXMOE_V2P(QT_I8, 0)
    MXMOE_V2P(QT_I8, 1)
    MXMOE_V2P(QT_I4, 0)
    MXMOE_V2P(QT_I4, 1)
    MXMOE_V2P(QT_F16, 0)
    MXMOE_V2P(QT_F16, 1)
    MXMOE_V2P(QT_F16, 2)
    MXMOE_V2P(QT_BF16, 0)
    MXMOE_V2P(QT_BF16, 1)
    MXMOE_V2P(QT_BF16, 2)
#undef MXMOE_V2P
    if (!done && !family(qt)) {  // the other tile bodies (their own prologue / LDS use; never prefetched into)
      PTile cur;
      p_resolve(args, idx, cur);
      const SplitK& sk = cur.sk;
      if ((QM & (1 << QT_I4G)) && qt == QT_I4G) {
        if (cls == 0) gg_tile_g128<V2Cfg<256>>(cur.mt, cur.A, cur.B, cur.SA, cur.SB, cur.C, cur.m0, cur.n0, lds);
        else gg_tile_g128<V2Cfg<128>>(cur.mt, cur.A, cur.B, cur.SA, cur.SB, cur.C, cur.m0, cur.n0, lds);
      } else if ((QM & (1 << QT_F8)) && qt == QT_F8) {
        if (cls == 0) gg_tile_v2<V2Cfg<256>, QT_F8, 0>(cur.mt, cur.A, cur.B, cur.SA, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else gg_tile_v2<V2Cfg<128>, QT_F8, 0>(cur.mt, cur.A, cur.B, cur.SA, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
      } else if ((QM & (1 << QT_W4A16)) && qt == QT_W4A16) {
        if (cls == 0) gg_tile_wo<WoCfg<256>, 4>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 4>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else gg_tile_wo<WoCfg<64, 1>, 4>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
      } else if ((QM & (1 << QT_W8A16)) && qt == QT_W8A16) {
        if (cls == 0) gg_tile_wo<WoCfg<256>, 8>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 8>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else gg_tile_wo<WoCfg<64, 1>, 8>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
      } else if ((QM & (1 << QT_W2A16)) && qt == QT_W2A16) {
        if (cls == 0) gg_tile_wo<WoCfg<256>, 2>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else if (cls == 1) gg_tile_wo<WoCfg<128, 1>, 2>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
        else gg_tile_wo<WoCfg<64, 1>, 2>(cur.mt, cur.A, cur.B, cur.SB, cur.C, cur.m0, cur.n0, lds, sk);
      }
      __syncthreads();  // the body's LDS use ends for every wave before the next tile's DMA
    }
    pref = r.pref;
    s_prev = r.stores;
  }
}

}  // namespace mxmoe
