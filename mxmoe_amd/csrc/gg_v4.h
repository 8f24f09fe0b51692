// gg_v4.h — lab only (-DMXMOE_LAB): v4d, the 256 x 256 GroupGEMM tile at ONE wave per SIMD, built on
// v2x's LDS-DMA discipline.
//
// Why: v2x (gg_tile_v2, 8 waves of 128 x 64 at two waves per SIMD) reads 192 KiB of LDS fragments per
// 128-B K stage (8 waves x (128 + 64) rows x 128 B) for 2048 MFMA cycles per SIMD and runs ~2440
// cycles per stage. Four waves of 128 x 128 read 128 KiB for the same MFMA work, and one wave per
// SIMD gets 512 registers: 256 AGPRs hold the 128 x 128 int32 / f32 accumulators, the VGPRs hold two
// fragment sets (next K half read under the current half's MFMAs, counted lgkmcnt by the compiler).
//
// Mainloop (per wave, stage s = 128 B of K; one barrier per stage, placed in the MIDDLE of the
// second K half so MFMAs on registers run on both sides of it):
//   after barrier B(s-1):  read F0 <- (s, half 0)          | MFMA on F1 rows FM/2.. (s-1, half 1)
//                          LDS-DMA A(s+1) (8 pieces)        |
//                          read F1 <- (s, half 1)          | MFMA on F0, all rows
//                          LDS-DMA B(s+2) (8 pieces)        |
//                                                            MFMA on F1 rows 0..FM/2 (s, half 1)
//   wait vmcnt(GB) (A(s+1) and B(s+1) landed, B(s+2) may fly), barrier B(s).
// LDS image = v2x's (A ring of 2 stages, B ring of 3; 128-B rows, (row >> 1) & 7 chunk swizzle
// applied to the DMA source and to the reads); buffer-form DMA with out-of-range rows / K-tail
// chunks read as zeros. Ring safety: A(s+1) refills the A slot of stage s-1 and B(s+2) the B slot
// of stage s-1, issued after B(s-1), which every wave reaches only once its reads of stage s-1
// have been consumed by MFMAs. Accumulation order per output: K stages in order, half 0 then half
// 1 (as every other body): bit-identical int32 sums, identical f32 sums to v2x's order.
// Epilogue: epilogue_v3 (scales, fp16 rounding, per-wave LDS staging of the 128 x 128 sub-tile
// in the drained ring, 16-B row stores; optional fused SiLU).
#pragma once

#include "gg_device.h"

namespace mxmoe {

template <int BM_>
struct V4Cfg {
  static constexpr int BM = BM_, BN = 256, NT = 256, BKB = 128, WM = 2, WN = 2;
  static constexpr int WTM = BM / WM, WTN = BN / WN;  // 128 x 128 (BM 256), 64 x 128, 32 x 128
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int SLOT = 256 * BKB;               // ring slots sized for 256 rows (32 KiB)
  static constexpr int GA = BM / 32, GB = BN / 32;     // 8-row x 128-B DMA pieces per wave per stage
  static constexpr int LDS_BYTES = 5 * SLOT;           // A ring (2) + B ring (3) = 160 KiB
  static_assert(FM % 2 == 0, "the second K half is split by fragment rows around the barrier");
  static_assert(WM * WN * WTM * WTN * 2 <= LDS_BYTES, "the epilogue staging fits the drained ring");
  static_assert(FM * FN * NT * 16 <= SPLITK_SLAB_BYTES, "split-K slab");
};

template <class Cfg>
struct V4Frag {
  v4i a[Cfg::FM];
  v4i b[Cfg::FN];
};
template <class Cfg>
__device__ __forceinline__ void v4_read(V4Frag<Cfg>& f, const uint8_t* As, const uint8_t* Bs, uint32_t off) {
#pragma unroll
  for (int i = 0; i < Cfg::FM; ++i) f.a[i] = *reinterpret_cast<const v4i*>(As + i * 2048 + off);
#pragma unroll
  for (int j = 0; j < Cfg::FN; ++j) f.b[j] = *reinterpret_cast<const v4i*>(Bs + j * 2048 + off);
}
// MFMAs of fragment rows [I0, I1) of one K half, all columns (operands swapped: src0 = B, so a lane
// owns 4 consecutive output columns, the layout epilogue_v3 packs)
template <class Cfg, int QT, int I0, int I1>
__device__ __forceinline__ void v4_mma(const V4Frag<Cfg>& f, typename AccT<QT>::type (&acc)[Cfg::FM][Cfg::FN]) {
#pragma unroll
  for (int i = I0; i < I1; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::FN; ++j) {
      if constexpr (QT == QT_I8) {
        acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.b[j], f.a[i], acc[i][j], 0, 0, 0);
      } else {
        static_assert(QT == QT_F16, "v4d: fp16 and w8a8 bodies");
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, f.b[j]), __builtin_bit_cast(v8h, f.a[i]),
                                                           acc[i][j], 0, 0, 0);
      }
    }
}

template <class Cfg, int QT>
__device__ __forceinline__ void gg_tile_v4(const GGMeta& mt, const uint8_t* __restrict__ A,
                                           const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                           const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0, int n0,
                                           uint8_t* lds, const SplitK& sk) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB, H = FM / 2;
  typedef typename AccT<QT>::type acc_t;
  typedef V4Frag<Cfg> Frag;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N, kbytes = mt.kbytes;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = sk.nst, ks0 = sk.ks0;

  // per-tile buffer resources (rows past M / N read as zeros) and fixed 32-bit lane offsets
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(A) + (int64_t)m0 * lda, (short)0, (int)(min(M - m0, Cfg::BM) * lda), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(B) + (int64_t)n0 * ldb, (short)0, (int)(min(N - n0, Cfg::BN) * ldb), 0x00020000);
  uint32_t voA[GA], voB[GB];
  int kcA[GA], kcB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      kcA[j] = (p ^ ((row >> 1) & 7)) << 4;
      voA[j] = (uint32_t)(row * lda) + kcA[j];
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      kcB[j] = (p ^ ((row >> 1) & 7)) << 4;
      voB[j] = (uint32_t)(row * ldb) + kcB[j];
    }
  }
  uint8_t* const ringA = lds;
  uint8_t* const ringB = lds + 2 * Cfg::SLOT;
  auto dma_a = [&](int t, bool full) {
    const int kb = (ks0 + t) * Cfg::BKB;
    uint8_t* dst = ringA + (t & 1) * Cfg::SLOT;
#pragma unroll
    for (int j = 0; j < GA; ++j)
      bdma16(rsA, dst + (wave * GA + j) * 1024, full || kb + kcA[j] < kbytes ? voA[j] : 0x80000000u, kb);
  };
  auto dma_b = [&](int t, bool full) {
    const int kb = (ks0 + t) * Cfg::BKB;
    uint8_t* dst = ringB + (t % 3) * Cfg::SLOT;
#pragma unroll
    for (int j = 0; j < GB; ++j)
      bdma16(rsB, dst + (wave * GB + j) * 1024, full || kb + kcB[j] < kbytes ? voB[j] : 0x80000000u, kb);
  };
  const int nst_full = (ks0 + nst) * Cfg::BKB > kbytes ? nst - 1 : nst;  // stages [0, nst_full) have no K tail
  auto full = [&](int t) { return t < nst_full; };

  acc_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc_t{0, 0, 0, 0};

  const int swz = (r16 >> 1) & 7;
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u, b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  const uint32_t off0 = (uint32_t)((g ^ swz) << 4), off1 = (uint32_t)(((4 + g) ^ swz) << 4);
  auto rd = [&](Frag& f, int t, uint32_t off) {
    v4_read<Cfg>(f, ringA + (t & 1) * Cfg::SLOT + a_row, ringB + (t % 3) * Cfg::SLOT + b_row, off);
  };

  if (nst > 0) {
    Frag F0, F1;
    dma_a(0, full(0));
    dma_b(0, full(0));
    if (nst > 1) {
      dma_b(1, full(1));
      wait_vmcnt<GB>();
    } else {
      wait_vmcnt<0>();
    }
    lds_barrier();  // B(-1): stage 0 landed for every wave
    // iteration 0 (no deferred rows yet)
    rd(F0, 0, off0);
    if (nst > 1) dma_a(1, full(1));
    v4_mma<Cfg, QT, 0, FM>(F0, acc);
    rd(F1, 0, off1);
    if (nst > 2) dma_b(2, full(2));
    v4_mma<Cfg, QT, 0, H>(F1, acc);
    if (nst > 2) wait_vmcnt<GB>();
    else wait_vmcnt<0>();
    lds_barrier();  // B(0)
    int s = 1;
    // steady state: A(s+1) and B(s+2) exist and are full stages; one basic block per stage
    const int nsteady = nst_full - 2;
    for (; s < nsteady; ++s) {
      // three segments fenced by sched_barrier (MFMAs would otherwise drift across the stage-end
      // barrier, which orders memory only): inside each, sched_group_barrier fixes the interleave
      constexpr int NR = FM + FN, S1 = H * FN, S2 = FM * FN;
      // (1) F0's reads two per MFMA of F1's deferred rows, the A pieces spread over the rest of them
      rd(F0, s, off0);
      v4_mma<Cfg, QT, H, FM>(F1, acc);
      dma_a(s + 1, true);
      {
        constexpr int R1 = (NR + 1) / 2 < S1 ? (NR + 1) / 2 : S1;
        constexpr int K1 = (S1 - R1) / GA, K1R = S1 - R1 - K1 * GA;
#pragma unroll
        for (int q = 0; q < R1; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
#pragma unroll
        for (int q = 0; q < GA; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, K1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, K1R, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // (2) F0's MFMAs with F1's reads early (one per 2 MFMAs) and the B pieces spread over the rest
      v4_mma<Cfg, QT, 0, FM>(F0, acc);
      rd(F1, s, off1);
      dma_b(s + 2, true);
      {
        constexpr int R2 = 2 * NR < S2 ? NR : S2 / 2;
        constexpr int K2 = (S2 - 2 * R2) / GB, K2R = S2 - 2 * R2 - K2 * GB;
#pragma unroll
        for (int q = 0; q < R2; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, NR - R2, 0);
#pragma unroll
        for (int q = 0; q < GB; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, K2, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, K2R, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      // (3) F1 rows 0..H, then the stage-end wait and barrier
      v4_mma<Cfg, QT, 0, H>(F1, acc);
      __builtin_amdgcn_sched_barrier(0);
      wait_vmcnt<GB>();
      lds_barrier();  // B(s)
    }
    for (; s < nst; ++s) {  // the last stages (K tail, no more pieces to issue)
      rd(F0, s, off0);
      v4_mma<Cfg, QT, H, FM>(F1, acc);
      if (s + 1 < nst) dma_a(s + 1, full(s + 1));
      v4_mma<Cfg, QT, 0, FM>(F0, acc);
      rd(F1, s, off1);
      if (s + 2 < nst) dma_b(s + 2, full(s + 2));
      v4_mma<Cfg, QT, 0, H>(F1, acc);
      if (s + 2 < nst) wait_vmcnt<GB>();
      else wait_vmcnt<0>();
      lds_barrier();  // B(s)
    }
    v4_mma<Cfg, QT, H, FM>(F1, acc);  // the deferred rows of the last stage
  } else {
    __syncthreads();
  }
  if (!splitk_reduce<Cfg::NT>(acc, sk, lds)) return;  // split-K: only the last slice writes C
  epilogue_v3<Cfg, QT>(mt, acc, SA, SB, C, m0, n0, lds);
}

template <int QM>
__global__ __launch_bounds__(256, 1) void gg_v4_kernel(GGArgs args) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[V4Cfg<256>::LDS_BYTES];
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const GGMeta mt = args.meta[td.prob];
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[td.prob]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[td.prob]);
  const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
  const _Float16* SB = static_cast<const _Float16*>(args.ptr_SB[td.prob]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[td.prob]);
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
    if (cls == 0) gg_tile_v4<V4Cfg<256>, QT_I8>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v4<V4Cfg<128>, QT_I8>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_F16)) && mt.qtype == QT_F16) {
    if (cls == 0) gg_tile_v4<V4Cfg<256>, QT_F16>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_v4<V4Cfg<128>, QT_F16>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v4<V4Cfg<64>, QT_F16>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  }
}

}  // namespace mxmoe
