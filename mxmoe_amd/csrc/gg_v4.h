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
__device__ __forceinline__ void v4_mma1(const V4Frag<Cfg>& f, int i, int j, typename AccT<QT>::type (&acc)[Cfg::FM][Cfg::FN]) {
  if constexpr (QT == QT_I8) {
    acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.b[j], f.a[i], acc[i][j], 0, 0, 0);
  } else {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, f.b[j]), __builtin_bit_cast(v8h, f.a[i]),
                                                       acc[i][j], 0, 0, 0);
  }
}

// int4 (w4a4): a 16-B fragment read holds 32 codes of one 64-B K half = two MFMA K steps (t = 0: words
// 0-1, t = 1: words 2-3, the same K map for A and B, as gg_tile_v3); each step's operands are the
// nibbles widened to 16 * q int8 (widen_i4: the int32 sum is exactly 256 * sum(a * b))
template <class Cfg>
struct V4Wide {
  v4i b[Cfg::FN];  // B fragments of one K step, widened
};
__device__ __forceinline__ v4i v4_widen(const v4i& raw, int t) { return widen_i4(v2i{raw[2 * t], raw[2 * t + 1]}); }
template <class Cfg>
__device__ __forceinline__ void v4_widen_b(const V4Frag<Cfg>& f, int t, V4Wide<Cfg>& w) {
#pragma unroll
  for (int j = 0; j < Cfg::FN; ++j) w.b[j] = v4_widen(f.b[j], t);
}
// one int4 K step of fragment row i (A widened here), all columns
template <class Cfg>
__device__ __forceinline__ void v4_mma_i4row(const V4Frag<Cfg>& f, const V4Wide<Cfg>& w, int t, int i,
                                             v4i (&acc)[Cfg::FM][Cfg::FN]) {
  const v4i aw = v4_widen(f.a[i], t);
#pragma unroll
  for (int j = 0; j < Cfg::FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(w.b[j], aw, acc[i][j], 0, 0, 0);
}
template <class Cfg>
__device__ __forceinline__ void v4_mma_i4(const V4Frag<Cfg>& f, int t, v4i (&acc)[Cfg::FM][Cfg::FN]) {
  V4Wide<Cfg> w;
  v4_widen_b<Cfg>(f, t, w);
#pragma unroll
  for (int i = 0; i < Cfg::FM; ++i) v4_mma_i4row<Cfg>(f, w, t, i, acc);
}

// Epilogue of the v4d tile: epilogue_v3's arithmetic and staging, with the tile's row / column
// scales read from the LDS stash (`sl`: SA of rows m0.. at [0, 256), SB of columns n0.. at [256, 512),
// clamped at load time) instead of global loads at the epilogue's start (their L2 / HBM latency was
// exposed at every tile boundary).
template <class Cfg, int QT>
__device__ __forceinline__ void epilogue_v4(const GGMeta& mt, typename AccT<QT>::type (&acc)[Cfg::FM][Cfg::FN],
                                            const _Float16* sl, _Float16* __restrict__ C, int m0, int n0, uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N;
  constexpr int RB = Cfg::WTN * 2, CPR = RB / 16;  // staged row bytes, 16-B chunks per row
  uint8_t* reg = lds + wave * (Cfg::WTM * Cfg::WTN * 2);
  const int mrow0 = m0 + wm * Cfg::WTM, ncol0 = n0 + wn * Cfg::WTN;
  uint2 sbw[FN];
  if constexpr (QT != QT_F16) {
#pragma unroll
    for (int j = 0; j < FN; ++j) sbw[j] = *reinterpret_cast<const uint2*>(sl + 256 + wn * Cfg::WTN + j * 16 + 4 * g);
  }
  auto pack_frag = [&](int i, int j, _Float16 sai) {
    if constexpr (QT == QT_F16) return pack4_f16(acc[i][j]);
    else return scale_pack4<(QT == QT_I4) ? 8 : 0>(acc[i][j], sai, sbw[j]);
  };
  if ((mt.reserved2 & META_SILU) != 0) {  // fused SiLU (as gg_tile_v2): rows of WTN / 2 outputs
    constexpr int ORB = Cfg::WTN, OCPR = ORB / 16;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = i * 16 + r16;
      _Float16 sai = 0;
      if constexpr (QT != QT_F16) sai = sl[wm * Cfg::WTM + ml];
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
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int ml = i * 16 + r16;
    _Float16 sai = 0;
    if constexpr (QT != QT_F16) sai = sl[wm * Cfg::WTM + ml];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint2 pk = pack_frag(i, j, sai);
      const int q = 2 * j + (g >> 1);
      *reinterpret_cast<uint2*>(reg + ml * RB + ((q ^ (ml & (CPR - 1))) << 4) + (g & 1) * 8) = pk;
    }
  }
  constexpr int RPI = 64 / CPR;  // staged rows per wave-instruction
  _Float16* const cbase = C + (int64_t)mrow0 * mt.ldc + ncol0;  // wave-uniform
  const bool narrow = (int64_t)Cfg::WTM * mt.ldc < (int64_t)1 << 29;
#pragma unroll 4
  for (int it = 0; it < Cfg::WTM / RPI; ++it) {
    const int row = it * RPI + lane / CPR, q = lane % CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(reg + row * RB + ((q ^ (row & (CPR - 1))) << 4));
    const int m = mrow0 + row, n = ncol0 + q * 8;
    if (m < M && n < N) store_c16(cbase, (int64_t)row * mt.ldc + q * 8, narrow, v);
  }
}

// OPT & 1: in-kernel s_memtime stamps of the steady stages (diagnostics build: per wave the cycles of
// segments 1 / 2 / 3, the stage-end vmcnt wait and the barrier, summed over the steady stages, into
// g_gg_stamp — slot (block, wave): {seg1, seg2, seg3, stages}, slot (block, wave + 4): {vm, bar, 0,
// stages}; tools/stamps_v4.py)
template <class Cfg, int QT, int OPT = 0>
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
  // int paths: this thread's row and column scale (one register across the mainloop), stashed in the
  // dead ring after it (past the 128-KiB epilogue image) for epilogue_v4
  constexpr int STASH = 128 * 1024;
  uint32_t sc_t = 0;  // SA | SB << 16
  if constexpr (qt_scaled(QT)) {
    const uint16_t a = __builtin_bit_cast(uint16_t, SA[min(m0 + min(tid, Cfg::BM - 1), M - 1)]);
    const uint16_t b = __builtin_bit_cast(uint16_t, SB[min(n0 + tid, N - 1)]);
    sc_t = (uint32_t)a | ((uint32_t)b << 16);
  }

  const int swz = (r16 >> 1) & 7;
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u, b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  const uint32_t off0 = (uint32_t)((g ^ swz) << 4), off1 = (uint32_t)(((4 + g) ^ swz) << 4);
  auto rd = [&](Frag& f, int t, uint32_t off) {
    v4_read<Cfg>(f, ringA + (t & 1) * Cfg::SLOT + a_row, ringB + (t % 3) * Cfg::SLOT + b_row, off);
  };

  // the three MFMA parts of a stage (int8 / fp16: all rows of half 0, then rows 0..H of half 1 before
  // the stage-end barrier and rows H..FM after it; int4: both K steps of half 0, then step 0 of half 1
  // before the barrier and step 1 after it)
  auto mma_all = [&](const Frag& f) {
    if constexpr (QT == QT_I4) {
      v4_mma_i4<Cfg>(f, 0, acc);
      v4_mma_i4<Cfg>(f, 1, acc);
    } else {
      v4_mma<Cfg, QT, 0, FM>(f, acc);
    }
  };
  auto mma_first = [&](const Frag& f) {
    if constexpr (QT == QT_I4) v4_mma_i4<Cfg>(f, 0, acc);
    else v4_mma<Cfg, QT, 0, H>(f, acc);
  };
  auto mma_second = [&](const Frag& f) {
    if constexpr (QT == QT_I4) v4_mma_i4<Cfg>(f, 1, acc);
    else v4_mma<Cfg, QT, H, FM>(f, acc);
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
    mma_all(F0);
    rd(F1, 0, off1);
    if (nst > 2) dma_b(2, full(2));
    mma_first(F1);
    if (nst > 2) wait_vmcnt<GB>();
    else wait_vmcnt<0>();
    lds_barrier();  // B(0)
    int s = 1;
    // steady state: A(s+1) and B(s+2) exist and are full stages; one basic block per stage
    const int nsteady = nst_full - 2;
    // steady state, hand-chunked (OPT & 1, the default build): every chunk is fenced by
    // sched_barrier(0), so the interleave of reads, MFMAs and DMA pieces is fixed in program order
    // (left to sched_group_barrier, hipcc bunched the int8 body's B pieces and F1 reads at the end of
    // the second segment: the reads' latency and 8 back-to-back DMA issues exposed before the barrier)
    //   seg 1 (C1 = 8 chunks):  2 reads of F0 (B fragments first, then A) | S1 / C1 MFMAs of F1's deferred
    //                          rows | 1 A piece per C1 / GA chunks
    //   seg 2 (C2 = 16 chunks): 1 read of F1 (B, then the A rows seg 3 needs, then the rest) | S2 / C2
    //                          MFMAs of F0, row-major | 1 B piece per C2 / GB chunks
    //   seg 3: F1 rows 0..H, then the stage-end wait and barrier
    constexpr int NR = FM + FN, S1 = H * FN, S2 = FM * FN, C1 = 8, C2 = 16;
    static_assert(S1 % C1 == 0 && S2 % C2 == 0 && C1 % GA == 0 && C2 % GB == 0, "v4d chunking");
    const uint8_t* const a0 = ringA + a_row;
    const uint8_t* const b0 = ringB + b_row;
    uint64_t st_seg[3] = {0, 0, 0}, st_vm = 0, st_bar = 0;
    if constexpr (QT == QT_I4) {
      // int4 steady stage: 256 MFMAs (4 K steps x 64) and 384 widening VALU per wave, hand-chunked so
      // every widened B set is built a chunk row ahead of its first MFMA:
      //   seg 1 (8 chunks, one fragment row each): F1 step 1 (A widened per row, B set wb1 built in
      //          seg 3) | F0's 16 reads, 2 per chunk | F0's B step 0 widened in chunks 4-7 | A pieces
      //   seg 2 (16 chunks: step 0 rows, then step 1 rows of F0) | F1's 16 reads, 1 per chunk | F0's B
      //          step 1 widened in chunks 0-7, F1's B step 0 in chunks 8-15 | B pieces
      //   seg 3 (8 chunks): F1 step 0 | F1's B step 1 widened, 1 per chunk; then wait + barrier
      // (written for the 256-row tile; the 128-row class runs every stage through the plain loop below)
      if constexpr (FM == 8 && FN == 8 && GA == 8 && GB == 8) {
      // one widened B set live at a time (register pressure: the pre-widened variant kept 2-3 sets and
      // hipcc shuffled accumulators through the AGPRs, 340 v_accvgpr moves per stage): each K-step
      // block widens its 8 B fragments at its start, then row by row (A widened per row, 8 MFMAs)
      V4Wide<Cfg> w;
      for (; s < nsteady; ++s) {
        const uint8_t* As = a0 + (s & 1) * Cfg::SLOT;
        const uint8_t* Bs = b0 + (s % 3) * Cfg::SLOT;
        auto rd1 = [&](Frag& f, int k, uint32_t off) {
          if (k < FN) f.b[k] = *reinterpret_cast<const v4i*>(Bs + k * 2048 + off);
          else f.a[k - FN] = *reinterpret_cast<const v4i*>(As + (k - FN) * 2048 + off);
        };
        const int kb_a = (ks0 + s + 1) * Cfg::BKB, kb_b = (ks0 + s + 2) * Cfg::BKB;
        uint8_t* const da = ringA + ((s + 1) & 1) * Cfg::SLOT + wave * GA * 1024;
        uint8_t* const db = ringB + ((s + 2) % 3) * Cfg::SLOT + wave * GB * 1024;
        // seg 1: F1 step 1 (the deferred block) | F0's 16 reads | A pieces
        v4_widen_b<Cfg>(F1, 1, w);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          rd1(F0, 2 * c, off0);
          rd1(F0, 2 * c + 1, off0);
          v4_mma_i4row<Cfg>(F1, w, 1, c, acc);
          bdma16(rsA, da + c * 1024, voA[c], kb_a);
          __builtin_amdgcn_sched_barrier(0);
        }
        // seg 2: F0 steps 0 and 1 | F1's 16 reads | B pieces
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          v4_widen_b<Cfg>(F0, t, w);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            rd1(F1, 8 * t + c, off1);
            v4_mma_i4row<Cfg>(F0, w, t, c, acc);
            if ((c & 1) == 0) bdma16(rsB, db + (4 * t + (c >> 1)) * 1024, voB[4 * t + (c >> 1)], kb_b);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // seg 3: F1 step 0
        v4_widen_b<Cfg>(F1, 0, w);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v4_mma_i4row<Cfg>(F1, w, 0, c, acc);
          __builtin_amdgcn_sched_barrier(0);
        }
        wait_vmcnt<GB>();
        lds_barrier();  // B(s)
      }
      }
    } else
    for (; s < nsteady; ++s) {
      [[maybe_unused]] uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
      if constexpr ((OPT & 1) != 0) t0 = __builtin_amdgcn_s_memtime();
      const uint8_t* As = a0 + (s & 1) * Cfg::SLOT;
      const uint8_t* Bs = b0 + (s % 3) * Cfg::SLOT;
      auto rd1 = [&](Frag& f, int k, uint32_t off) {  // read k: B fragments 0..FN-1, then A 0..FM-1
        if (k < FN) f.b[k] = *reinterpret_cast<const v4i*>(Bs + k * 2048 + off);
        else f.a[k - FN] = *reinterpret_cast<const v4i*>(As + (k - FN) * 2048 + off);
      };
      const int kb_a = (ks0 + s + 1) * Cfg::BKB, kb_b = (ks0 + s + 2) * Cfg::BKB;
      uint8_t* const da = ringA + ((s + 1) & 1) * Cfg::SLOT + wave * GA * 1024;
      uint8_t* const db = ringB + ((s + 2) % 3) * Cfg::SLOT + wave * GB * 1024;
#pragma unroll
      for (int c = 0; c < C1; ++c) {
#pragma unroll
        for (int r = 0; r < (NR + C1 - 1) / C1; ++r)
          if (c * ((NR + C1 - 1) / C1) + r < NR) rd1(F0, c * ((NR + C1 - 1) / C1) + r, off0);
#pragma unroll
        for (int x = 0; x < S1 / C1; ++x) {
          const int idx = c * (S1 / C1) + x, i = H + idx / FN, j = idx % FN;
          v4_mma1<Cfg, QT>(F1, i, j, acc);
        }
        if (c % (C1 / GA) == 0) bdma16(rsA, da + (c / (C1 / GA)) * 1024, voA[c / (C1 / GA)], kb_a);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr ((OPT & 1) != 0) t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
      for (int c = 0; c < C2; ++c) {
        if (c < NR) rd1(F1, c, off1);
#pragma unroll
        for (int x = 0; x < S2 / C2; ++x) {
          const int idx = c * (S2 / C2) + x, i = idx / FN, j = idx % FN;
          v4_mma1<Cfg, QT>(F0, i, j, acc);
        }
        if (c % (C2 / GB) == 0) bdma16(rsB, db + (c / (C2 / GB)) * 1024, voB[c / (C2 / GB)], kb_b);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr ((OPT & 1) != 0) t2 = __builtin_amdgcn_s_memtime();
      v4_mma<Cfg, QT, 0, H>(F1, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((OPT & 1) != 0) t3 = __builtin_amdgcn_s_memtime();
      wait_vmcnt<GB>();
      if constexpr ((OPT & 1) != 0) t4 = __builtin_amdgcn_s_memtime();
      lds_barrier();  // B(s)
      if constexpr ((OPT & 1) != 0) {
        const uint64_t t5 = __builtin_amdgcn_s_memtime();
        st_seg[0] += t1 - t0;
        st_seg[1] += t2 - t1;
        st_seg[2] += t3 - t2;
        st_vm += t4 - t3;
        st_bar += t5 - t4;
      }
    }
#ifdef MXMOE_LAB
    if constexpr ((OPT & 1) != 0) {
      if (lane == 0 && blockIdx.x < kStampBlocks && nsteady > 1) {
        uint64_t* o = g_gg_stamp + ((size_t)blockIdx.x * 8 + wave) * 4;
        o[0] = st_seg[0];
        o[1] = st_seg[1];
        o[2] = st_seg[2];
        o[3] = (uint64_t)(nsteady - 1);
        uint64_t* o2 = g_gg_stamp + ((size_t)blockIdx.x * 8 + wave + 4) * 4;
        o2[0] = st_vm;
        o2[1] = st_bar;
        o2[2] = 0;
        o2[3] = (uint64_t)(nsteady - 1);
      }
    }
#endif
    for (; s < nst; ++s) {  // the last stages (K tail, no more pieces to issue)
      rd(F0, s, off0);
      mma_second(F1);
      if (s + 1 < nst) dma_a(s + 1, full(s + 1));
      mma_all(F0);
      rd(F1, s, off1);
      if (s + 2 < nst) dma_b(s + 2, full(s + 2));
      mma_first(F1);
      if (s + 2 < nst) wait_vmcnt<GB>();
      else wait_vmcnt<0>();
      lds_barrier();  // B(s)
    }
    mma_second(F1);  // the deferred part of the last stage
  } else {
    __syncthreads();
  }
  _Float16* const sl = reinterpret_cast<_Float16*>(lds + STASH);
  if constexpr (qt_scaled(QT)) {
    reinterpret_cast<uint16_t*>(sl)[tid] = (uint16_t)sc_t;  // (the ring is drained: every wave passed the
    reinterpret_cast<uint16_t*>(sl)[256 + tid] = (uint16_t)(sc_t >> 16);  // last stage's barrier)
  }
  if (!splitk_reduce<Cfg::NT>(acc, sk, lds)) return;  // split-K: only the last slice writes C
  if constexpr (qt_scaled(QT)) __syncthreads();        // the stash is visible to every wave
  epilogue_v4<Cfg, QT>(mt, acc, sl, C, m0, n0, lds);
}

// v4d's int4 (w4a4) tile, ONE fragment set (the int4 body of gg_tile_v4 kept two sets plus widened
// operands and hipcc spilled its steady loop into the AGPRs). A 64-B K half of a fragment holds two
// MFMA K steps (t = 0, 1; V4Wide / v4_widen as above). Per K half: step 0 — widen the 8 B fragments,
// then row by row widen A and run 8 MFMAs; step 1 — widen B again (words 2-3), and as each raw
// fragment is consumed the NEXT half's read goes into its registers (B reads at the step's start, the
// A read of row i after row i's MFMAs), so the reads of the next half run under this step's 64 MFMAs.
// One barrier per stage, between the second half's two steps: every wave has consumed all its reads of
// stage s there (the step-0 widening waited for them), and stage s+1 must have landed before the
// step-1 reads of its first half. LDS-DMA (v2x's image and buffer form, as gg_tile_v4): B(s+2) one
// piece per row of stage s's first step (its slot last held stage s-1, free since B(s-1)); A(s+2)
// one per row of the post-barrier step (its slot held stage s). At B(s): vmcnt(GB) leaves B(s+2) in
// flight; A(s+1) was issued a whole stage (4096 MFMA cycles) before.
template <class Cfg, int OPT = 0>
__device__ __forceinline__ void gg_tile_v4_i4(const GGMeta& mt, const uint8_t* __restrict__ A,
                                              const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                              const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0,
                                              int n0, uint8_t* lds, const SplitK& sk) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB;
  static_assert(GA % FM == 0 || FM % GA == 0, "A pieces per row");
  typedef V4Frag<Cfg> Frag;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N, kbytes = mt.kbytes;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = sk.nst, ks0 = sk.ks0;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(A) + (int64_t)m0 * lda, (short)0, (int)(min(M - m0, Cfg::BM) * lda), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(B) + (int64_t)n0 * ldb, (short)0, (int)(min(N - n0, Cfg::BN) * ldb), 0x00020000);
  uint32_t voA[GA], voB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      voA[j] = (uint32_t)(row * lda) + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      voB[j] = (uint32_t)(row * ldb) + ((p ^ ((row >> 1) & 7)) << 4);
    }
  }
  auto kc_of = [&](int G, int j) { return ((lane & 7) ^ ((((wave * G + j) * 8 + (lane >> 3)) >> 1) & 7)) << 4; };
  uint8_t* const ringA = lds;
  uint8_t* const ringB = lds + 2 * Cfg::SLOT;
  const int nst_full = (ks0 + nst) * Cfg::BKB > kbytes ? nst - 1 : nst;
  // piece j of operand A / B of stage t (`full`: no K-tail lanes)
  auto pa = [&](int t, int j, bool full) {
    const int kb = (ks0 + t) * Cfg::BKB;
    bdma16(rsA, ringA + (t & 1) * Cfg::SLOT + (wave * GA + j) * 1024,
           full || kb + kc_of(GA, j) < kbytes ? voA[j] : 0x80000000u, kb);
  };
  auto pb = [&](int t, int j, bool full) {
    const int kb = (ks0 + t) * Cfg::BKB;
    bdma16(rsB, ringB + (t % 3) * Cfg::SLOT + (wave * GB + j) * 1024,
           full || kb + kc_of(GB, j) < kbytes ? voB[j] : 0x80000000u, kb);
  };

  v4i acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  constexpr int STASH = 128 * 1024;
  uint32_t sc_t;
  {
    const uint16_t a = __builtin_bit_cast(uint16_t, SA[min(m0 + min(tid, Cfg::BM - 1), M - 1)]);
    const uint16_t b = __builtin_bit_cast(uint16_t, SB[min(n0 + tid, N - 1)]);
    sc_t = (uint32_t)a | ((uint32_t)b << 16);
  }
  const int swz = (r16 >> 1) & 7;
  const uint32_t a_row = (uint32_t)(wm * Cfg::WTM + r16) * 128u, b_row = (uint32_t)(wn * Cfg::WTN + r16) * 128u;
  const uint32_t offh[2] = {(uint32_t)((g ^ swz) << 4), (uint32_t)(((4 + g) ^ swz) << 4)};
  auto a_src = [&](int t, int h, int i) { return ringA + (t & 1) * Cfg::SLOT + a_row + i * 2048 + offh[h]; };
  auto b_src = [&](int t, int h, int j) { return ringB + (t % 3) * Cfg::SLOT + b_row + j * 2048 + offh[h]; };

  if (nst > 0) {
    Frag F;
    V4Wide<Cfg> w;
    pa(0, 0, nst_full > 0);
    for (int j = 1; j < GA; ++j) pa(0, j, nst_full > 0);
    for (int j = 0; j < GB; ++j) pb(0, j, nst_full > 0);
    if (nst > 1) {
      for (int j = 0; j < GB; ++j) pb(1, j, nst_full > 1);
      wait_vmcnt<GB>();
    } else {
      wait_vmcnt<0>();
    }
    lds_barrier();  // B(-1): stage 0 landed
#pragma unroll
    for (int j = 0; j < FN; ++j) F.b[j] = *reinterpret_cast<const v4i*>(b_src(0, 0, j));
#pragma unroll
    for (int i = 0; i < FM; ++i) F.a[i] = *reinterpret_cast<const v4i*>(a_src(0, 0, i));
    if (nst > 1)
      for (int j = 0; j < GA; ++j) pa(1, j, nst_full > 1);  // A(1): its slot is free (never used)
    // one K step of the current half: B widened, then rows; `nx` (next half's reads) go into the
    // registers each fragment frees: t = 1 only
    auto step = [&](int t, bool reads, int rt, int rh, int dma, int ds) __attribute__((always_inline)) {
      // dma: 0 none, 1 = B pieces of stage ds (one per row), 2 = A pieces of stage ds
      v4_widen_b<Cfg>(F, t, w);
      if (reads) {
#pragma unroll
        for (int j = 0; j < FN; ++j) F.b[j] = *reinterpret_cast<const v4i*>(b_src(rt, rh, j));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        v4_mma_i4row<Cfg>(F, w, t, i, acc);
        if (reads) F.a[i] = *reinterpret_cast<const v4i*>(a_src(rt, rh, i));
        if (dma == 1) {
#pragma unroll
          for (int q = i * GB / FM; q < (i + 1) * GB / FM; ++q) pb(ds, q, ds < nst_full);
        } else if (dma == 2) {
#pragma unroll
          for (int q = i * GA / FM; q < (i + 1) * GA / FM; ++q) pa(ds, q, ds < nst_full);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    int s = 0;
    const int nsteady = nst - 2;  // stages whose B(s+2) / A(s+2) exist (the K tail: `full` per stage)
    for (; s < nsteady; ++s) {
      step(0, false, 0, 0, 1, s + 2);  // half 0, step 0 | B(s+2)
      step(1, true, s, 1, 0, 0);       // half 0, step 1 | reads of half 1
      step(0, false, 0, 0, 0, 0);      // half 1, step 0
      wait_vmcnt<GB>();
      lds_barrier();                   // B(s)
      step(1, true, s + 1, 0, 2, s + 2);  // half 1, step 1 | reads of stage s+1 half 0 | A(s+2)
    }
    for (; s < nst; ++s) {  // the last two stages (no more pieces)
      step(0, false, 0, 0, 0, 0);
      step(1, true, s, 1, 0, 0);
      step(0, false, 0, 0, 0, 0);
      wait_vmcnt<0>();
      lds_barrier();
      if (s + 1 < nst) step(1, true, s + 1, 0, 0, 0);
      else step(1, false, 0, 0, 0, 0);
    }
  } else {
    __syncthreads();
  }
  _Float16* const sl = reinterpret_cast<_Float16*>(lds + STASH);
  reinterpret_cast<uint16_t*>(sl)[tid] = (uint16_t)sc_t;
  reinterpret_cast<uint16_t*>(sl)[256 + tid] = (uint16_t)(sc_t >> 16);
  if (!splitk_reduce<Cfg::NT>(acc, sk, lds)) return;
  __syncthreads();
  epilogue_v4<Cfg, QT_I4>(mt, acc, sl, C, m0, n0, lds);
}

template <int QM, int OPT = 0>
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
    if (cls == 0) gg_tile_v4<V4Cfg<256>, QT_I8, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v4<V4Cfg<128>, QT_I8, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_I4)) && mt.qtype == QT_I4) {
    if (cls == 0) gg_tile_v4_i4<V4Cfg<256>, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v4_i4<V4Cfg<128>, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  } else if ((QM & (1 << QT_F16)) && mt.qtype == QT_F16) {
    if (cls == 0) gg_tile_v4<V4Cfg<256>, QT_F16, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else if (cls == 1) gg_tile_v4<V4Cfg<128>, QT_F16, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
    else gg_tile_v4<V4Cfg<64>, QT_F16, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds, sk);
  }
}

}  // namespace mxmoe
