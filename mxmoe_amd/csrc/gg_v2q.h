// gg_v2q.h — v2q: the persistent v2x whose tile boundary costs no MFMA time it can hide.
//
// What it replaces (reference, read as text): the fused persistent kernel's tile loop
// (compose_kernel.py:150-224, tile_scheduler.cuh:25-50) with the per-tile mainloop
// cta_gemm.cuh:423-608 and epilogue mm_tile.cuh:610-662 — same arithmetic as gg_tile_v2.
//
// Why: with one 160-KiB workgroup per CU, a v2x tile boundary is a serial
// chain — epilogue (pack to LDS, read back, 128 KiB of stores: 3.4-4.4 us), block retire + dispatch
// (~1.5 us), prologue (stage 0's LDS-DMA latency) — during which the CU's matrix pipes idle: ~20 %
// of a w8a8 layer call. v2q keeps one workgroup per CU walking a planned tile list (the v2p table,
// [k][workgroup]) and reorders the boundary:
//   * after tile i's last barrier the whole LDS ring is free: the early waves issue tile i+1's
//     A0, B0, B1, A1, B2 (every ring slot, ~160 KiB) FIRST;
//   * then every wave stores tile i's C straight from its accumulators (no LDS: pairs of 16 x 16
//     blocks exchanged by v_permlane16_swap, one 16-B buffer store per lane and block pair);
//   * tile i+1 waits only for A0 / B0 (counted vmcnt: its later prefetch pieces and tile i's stores
//     stay in flight) and its first iteration issues no DMA; the stores must drain before iteration
//     1's DMA, i.e. within two stages.
// The mainloop is v2x's (staggered SIMD partners, 3-stage B ring, buffer-form LDS-DMA spread one
// piece per 4 MFMAs, issued by waves 0-3 for their partners too; int4 tiles per wave).
#pragma once

#include "gg_device.h"

namespace mxmoe {

// LDS map (as v2x with V2_B3): A slots [0, 32K) [32K, 64K); B ring [64K, 96K) [96K, 128K) [128K, 160K)
constexpr int Q_ASLOT = 32768, Q_BBASE = 65536, Q_BSLOT = 32768;
// C store cache policy (template SAUX): 16 = sc1 (write-once lines leave the XCD's L2; v2x's
// choice), 0 = plain. tools/store_probe.hip: a 128-KiB tile drains in 1366 (plain) vs 2434 (sc1)
// cycles with 32 CUs storing.

// What a tile leaves in flight for the next one (per wave: the counts differ between early and
// late waves): `pref` the next tile's ring was filled by the previous tile, `after` LDS-DMA pieces
// this wave issued after the next tile's A0 / B0, `stores` C stores this wave issued after those.
struct QState {
  bool pref;
  int after;
  int stores;
};

// s_waitcnt vmcnt(c) for the largest c of a short ladder with c <= n (n wave-uniform): waits for at
// least the operations vmcnt(n) would (never fewer: correct), at most a few more
__device__ __forceinline__ void q_wait_le(int n) {
  if (n >= 40) wait_vmcnt<40>();
  else if (n >= 32) wait_vmcnt<32>();
  else if (n >= 24) wait_vmcnt<24>();
  else if (n >= 20) wait_vmcnt<20>();
  else if (n >= 16) wait_vmcnt<16>();
  else if (n >= 12) wait_vmcnt<12>();
  else if (n >= 8) wait_vmcnt<8>();
  else if (n >= 4) wait_vmcnt<4>();
  else wait_vmcnt<0>();
}

__device__ __forceinline__ bool q_edma(int qt) { return qt != QT_I4; }  // int4 tiles: per-wave issue

// One operand's pieces of one 128-B K stage into `dst`: rows of G x 8 per wave; EDMA: the early
// waves issue their partner's (w + 4) rows too, the late waves none. Rows past the buffer's range
// (num_records) and K-tail chunks past `kbytes` read as zeros. Returns the pieces this wave issued.
__device__ __forceinline__ int q_dma(const __amdgpu_buffer_rsrc_t& rs, int G, int64_t ld, int kb, int kbytes,
                                     bool edma, int wave, int lane, uint8_t* dst) {
  const bool early = wave < 4;
  if (edma && !early) return 0;
  const int rsub = lane >> 3, p = lane & 7;
  const bool full = kb + 128 <= kbytes;
  int n = 0;
#pragma unroll
  for (int w2 = 0; w2 < 2; ++w2) {
    if (w2 == 1 && !edma) break;
    const int ww = wave + w2 * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= G) break;
      const int row = (ww * G + j) * 8 + rsub;  // the partner's rows: + 8 G HALFW, same swizzle
      const int kc = (p ^ (((wave * G + j) * 8 + rsub) >> 1 & 7)) << 4;
      const uint32_t vo = (uint32_t)(row * ld) + (uint32_t)kc;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + (ww * G + j) * 1024), 16,
                                               (full || kb + kc < kbytes) ? vo : 0x80000000u, kb, 0, 0);
      ++n;
    }
  }
  return n;
}

// The ring fill of tile `t`, issued by the early waves for every quant type (each issues its
// partner's rows too): head = A0, B0, B1, tail = A1, B2 (as far as the tile has stages). In that
// order "A0 and B0 landed" is vmcnt(pieces issued after them). q_fill_head returns {pieces in
// all, pieces after A0 / B0}; q_fill_tail the pieces it issued (this wave's counts).
struct QFillSrc {
  __amdgpu_buffer_rsrc_t a, b;
  int GA, nst, kb0;
};
__device__ __forceinline__ QFillSrc q_fill_src(const PTile& t) {
  const GGMeta& m = t.mt;
  const int bm = t.cls == 0 ? 256 : t.cls == 1 ? 128 : 64;
  QFillSrc f;
  f.a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(t.A) + (int64_t)t.m0 * m.lda_b, (short)0,
                                          (int)(min(m.M - t.m0, bm) * m.lda_b), 0x00020000);
  f.b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(t.B) + (int64_t)t.n0 * m.ldb_b, (short)0,
                                          (int)(min(m.N - t.n0, 256) * m.ldb_b), 0x00020000);
  f.GA = bm / 64;
  f.nst = t.sk.nst;
  f.kb0 = t.sk.ks0 * 128;
  return f;
}
__device__ __forceinline__ int2 q_fill_head(const PTile& t, uint8_t* lds, int wave, int lane, bool edma) {
  const GGMeta& m = t.mt;
  const QFillSrc f = q_fill_src(t);
  if (f.nst <= 0) return int2{0, 0};
  int first = q_dma(f.a, f.GA, m.lda_b, f.kb0, m.kbytes, edma, wave, lane, lds);
  first += q_dma(f.b, 4, m.ldb_b, f.kb0, m.kbytes, edma, wave, lane, lds + Q_BBASE);
  const int after = f.nst > 1 ? q_dma(f.b, 4, m.ldb_b, f.kb0 + 128, m.kbytes, edma, wave, lane, lds + Q_BBASE + Q_BSLOT) : 0;
  return int2{first + after, after};
}
__device__ __forceinline__ int q_fill_tail(const PTile& t, uint8_t* lds, int wave, int lane, bool edma) {
  const GGMeta& m = t.mt;
  const QFillSrc f = q_fill_src(t);
  int n = 0;
  if (f.nst > 1) n += q_dma(f.a, f.GA, m.lda_b, f.kb0 + 128, m.kbytes, edma, wave, lane, lds + Q_ASLOT);
  if (f.nst > 2) n += q_dma(f.b, 4, m.ldb_b, f.kb0 + 256, m.kbytes, edma, wave, lane, lds + Q_BBASE + 2 * Q_BSLOT);
  return n;
}

template <class Cfg, int QT, int TRACE = 0, int SAUX = 16, int FILLALL = 0>
__device__ __forceinline__ QState gg_tile_v2q(const GGArgs& args, int cur_idx, int nx_idx, QState st, uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB;
  typedef typename AccT<QT>::type acc_t;
  typedef V2Half<Cfg, QT, 0> Half;
  constexpr bool EDMA = QT != QT_I4;
  constexpr int HALFW = 4;
  constexpr int NH = Half::kMfma, NR = Half::kReads, ND = GA + GB;
  constexpr int NDE = EDMA ? 2 * ND : ND;
  constexpr int KSE = 4 * NDE <= NH ? 4 : (NH / NDE > 0 ? NH / NDE : 1);
  constexpr int RESTE = NH - KSE * NDE > 0 ? NH - KSE * NDE : 0;
  static_assert(Cfg::WM * Cfg::WN == 8 && Cfg::BN == 256, "v2q: the 8-wave 256-column v2 tiles");
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // per tile: nothing lane-derived is hoisted out of the persistent loop
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const bool early = wave < HALFW;
  const int pw = EDMA ? (early ? 2 : 0) : 1;  // pieces this wave issues per (operand, row group)
  PTile t;
  p_resolve(args, cur_idx, t);
  const GGMeta& mt = t.mt;
  const int kbytes = mt.kbytes;
  const int nst = t.sk.nst, ks0 = t.sk.ks0;
  const int M = mt.M, N = mt.N;

  auto abuf = [&](int s) { return lds + (s & 1) * Q_ASLOT; };
  auto bbuf = [&](int s) { return lds + Q_BBASE + (s % 3) * Q_BSLOT; };
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(t.A) + (int64_t)t.m0 * mt.lda_b, (short)0, (int)(min(M - t.m0, Cfg::BM) * mt.lda_b), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(t.B) + (int64_t)t.n0 * mt.ldb_b, (short)0, (int)(min(N - t.n0, Cfg::BN) * mt.ldb_b), 0x00020000);
  // steady-state pieces (full stages, compile-time counts): lane offsets fixed for the tile
  uint32_t voA[GA], voB[GB];
  {
    const int rsub = lane >> 3, p = lane & 7;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave * GA + j) * 8 + rsub;
      voA[j] = (uint32_t)(row * mt.lda_b) + ((p ^ ((row >> 1) & 7)) << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave * GB + j) * 8 + rsub;
      voB[j] = (uint32_t)(row * mt.ldb_b) + ((p ^ ((row >> 1) & 7)) << 4);
    }
  }
  auto dma_full = [&](const __amdgpu_buffer_rsrc_t& rs, const uint32_t* vo, int G, int64_t ld, int kb, uint8_t* dst) {
    if (EDMA && !early) return;
#pragma unroll
    for (int w2 = 0; w2 < (EDMA ? 2 : 1); ++w2) {
      const int ww = wave + w2 * HALFW;
      const uint32_t radd = (uint32_t)(w2 * 8 * G * HALFW * ld);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= G) break;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + (ww * G + j) * 1024), 16, vo[j] + radd, kb, 0, 0);
      }
    }
  };
  const int nst_full = (ks0 + nst) * Cfg::BKB > kbytes ? nst - 1 : nst;  // stages [0, nst_full) are full
  // iteration s (>= 1) issues A(s+1) and B(s+2)
  auto dma_iter = [&](int s) {
    if (s + 1 < nst) {
      if (s + 1 < nst_full) dma_full(rsA, voA, GA, mt.lda_b, (ks0 + s + 1) * Cfg::BKB, abuf(s + 1));
      else q_dma(rsA, GA, mt.lda_b, (ks0 + s + 1) * Cfg::BKB, kbytes, EDMA, wave, lane, abuf(s + 1));
    }
    if (s + 2 < nst) {
      if (s + 2 < nst_full) dma_full(rsB, voB, GB, mt.ldb_b, (ks0 + s + 2) * Cfg::BKB, bbuf(s + 2));
      else q_dma(rsB, GB, mt.ldb_b, (ks0 + s + 2) * Cfg::BKB, kbytes, EDMA, wave, lane, bbuf(s + 2));
    }
  };
  // stage-end wait of iteration s >= 1: A(s+1), B(s+1) landed, B(s+2) may stay in flight
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

  [[maybe_unused]] auto tmark = [&](int slot) {
    if constexpr (TRACE != 0) {
      if (tid == 0 && cur_idx < kTraceBlocks) g_gg_trace[cur_idx * 4 + slot] = __builtin_amdgcn_s_memrealtime();
    }
  };
  tmark(0);
  // ---- prologue: the ring fill (issued by the previous tile when st.pref), A0 / B0 landed ----
  if (nst > 0) {
    if (!st.pref) {
      st.after = q_fill_head(t, lds, wave, lane, !FILLALL).y + q_fill_tail(t, lds, wave, lane, !FILLALL);
      st.stores = 0;
    }
    q_wait_le(st.after + st.stores);
    lds_barrier();
    // iteration 0: A1 / B1 landed; B2 and the previous tile's stores may stay in flight
    // (early waves: the fill's B2 and this wave's stores of the previous tile may stay in flight;
    //  the late waves have no loads outstanding: the fill is the early waves')
    // (FILLALL: every wave issued its own fill pieces; the late waves then require B2 as well here,
    //  since their EDMA mainloop has no later wait)
    const int w0 = (nst > 2 ? (FILLALL ? (early ? GB : 0) : 2 * GB) : 0) + st.stores;
    Half fr;
    if (!early) {  // late waves: the second K half of every stage deferred past the next barrier
      hread(fr, 0, 0);
      hmma(fr);
      hread(fr, 0, 1);
      if constexpr (FILLALL != 0) q_wait_le(w0);  // (else: no loads of the late waves outstanding here)
      lds_barrier();
      int s = 1;
      for (; s < nst_full - 2; ++s) {
        dma_full(rsA, voA, GA, mt.lda_b, (ks0 + s + 1) * Cfg::BKB, abuf(s + 1));
        dma_full(rsB, voB, GB, mt.ldb_b, (ks0 + s + 2) * Cfg::BKB, bbuf(s + 2));
        hmma(fr);  // second half of stage s-1
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
        if constexpr (!EDMA) stage_wait(s);  // (EDMA: late waves issue no loads)
        lds_barrier();
      }
      for (; s < nst; ++s) {
        dma_iter(s);
        hmma(fr);
        hread(fr, s, 0);
        hmma(fr);
        hread(fr, s, 1);
        if constexpr (!EDMA) stage_wait(s);  // (EDMA: late waves issue no loads)
        lds_barrier();
      }
      hmma(fr);
    } else {  // early waves
      // (a compiler barrier: otherwise the two branches' identical first reads are hoisted into a
      // shared head, and the read-group schedule below grabs the next half's reads -> 29 VGPRs spilled)
      asm volatile("" ::: "memory");
      hread(fr, 0, 0);
      hmma(fr);
      hread(fr, 0, 1);
      hmma(fr);
      q_wait_le(w0);
      lds_barrier();
      int s = 1;
      for (; s < nst_full - 2; ++s) {
        hread(fr, s, 0);
        dma_full(rsA, voA, GA, mt.lda_b, (ks0 + s + 1) * Cfg::BKB, abuf(s + 1));
        dma_full(rsB, voB, GB, mt.ldb_b, (ks0 + s + 2) * Cfg::BKB, bbuf(s + 2));
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
        dma_iter(s);
        hread(fr, s, 0);
        hmma(fr);
        hread(fr, s, 1);
        hmma(fr);
        stage_wait(s);
        lds_barrier();
      }
    }
  } else {
    wait_vmcnt<0>();
    __syncthreads();
  }
  tmark(1);

  // ---- between the tiles: scale loads (int paths), the next tile's ring fill, then C ----
  // LDS after the last barrier: every slot free. Order per wave: scale loads; (early waves) the
  // next tile's A0 / B0 / B1 (head fill) into A slot 0 / B slots 0-1; C of this tile staged through
  // A slot 1 + B slot 2 (64 KiB: every wave half its sub-tile per pass, reading back only its own
  // region, so no barrier inside a pass) into registers; a barrier (every wave's staging reads
  // done); (early waves) the tail fill A1 / B2 into those slots; then every wave's WTM / 8 C stores.
  // The stores are the youngest operations: the next tile's first waits leave them in flight.
  int ci = __builtin_amdgcn_readfirstlane(cur_idx), ni = __builtin_amdgcn_readfirstlane(nx_idx);
  asm volatile("" : "+s"(ci), "+s"(ni));  // opaque: the resolves below reload (scalar loads)
  p_resolve(args, ci, t);
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
    for (int j = 0; j < FN; ++j) sbw[j] = __builtin_bit_cast(uint2, *(gu64_t*)(sb + min(ncol0 + j * 16 + 4 * e_g, Ne - 4)));
  }
  const int64_t ldc = t.mt.ldc;
  const bool narrow = (int64_t)Cfg::WTM * ldc < (int64_t)1 << 29;  // C byte offsets < 2^30
  const bool split = t.sk.nsplit > 1;
  QState nxt{false, 0, 0};
  int nfill = 0;  // head-fill pieces this wave issued (younger than the scale loads)
  PTile nx;
  if (ni >= 0 && narrow && !split && nst > 0 && p_resolve(args, ni, nx)) {
    const int q = nx.mt.qtype;
    if ((q == QT_F16 || q == QT_I8 || q == QT_I4 || q == QT_BF16) && nx.sk.nsplit <= 1 && nx.sk.nst > 0) {
      const int2 f = q_fill_head(nx, lds, wave, lane, !FILLALL);
      nxt.pref = true;
      nxt.after = f.y;
      nfill = f.x;
    }
  }
  if constexpr (qt_scaled(QT)) q_wait_le(nfill);
  if (split && !splitk_reduce<Cfg::NT>(acc, t.sk, lds, etid)) return QState{false, 0, 0};

  // staging: wave w's 8-KiB region, 64 rows x 128 B with the (row & 7) chunk swizzle
  constexpr int RP = Cfg::WTM / 2;  // rows per pass (two passes fill the 64-KiB staging area)
  static_assert(RP * 128 * 8 <= 2 * Q_ASLOT, "staging: two passes of the 64-KiB area");
  uint8_t* const reg = (wave < HALFW ? lds + Q_ASLOT : lds + Q_BBASE + 2 * Q_BSLOT) + (wave % HALFW) * (RP * 128);
  uint4 cv[Cfg::WTM / 8];  // this wave's sub-tile in store order: rows [8 it, 8 it + 8), 16 B per lane
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = pass * (FM / 2); i < (pass + 1) * (FM / 2); ++i) {
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
      cv[pass * (RP / 8) + it] = *reinterpret_cast<const uint4*>(reg + rl * 128 + ((q ^ (rl & 7)) << 4));
    }
  }
  lds_barrier();  // every wave's staging reads are done: A slot 1 / B slot 2 are free
  if (nxt.pref) nxt.after += q_fill_tail(nx, lds, wave, lane, !FILLALL);
  _Float16* const cbase = t.C + (int64_t)mrow0 * ldc + ncol0;  // wave-uniform
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(cbase, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int it = 0; it < Cfg::WTM / 8; ++it) {
    const int row = it * 8 + (e_lane >> 3), q = e_lane & 7;
    const int m = mrow0 + row, n = ncol0 + q * 8;
    const bool in = m < Me && n < Ne;  // N % 8 == 0: an 8-column group is all in or all out
    if (narrow) {
      typedef unsigned int v4u_ __attribute__((ext_vector_type(4)));
      const v4u_ d = {cv[it].x, cv[it].y, cv[it].z, cv[it].w};
      __builtin_amdgcn_raw_buffer_store_b128(d, rsC, in ? (int)(((int64_t)row * ldc + q * 8) * 2) : (int)0x80000000, 0,
                                             SAUX);
    } else if (in) {
      *reinterpret_cast<uint4*>(cbase + (int64_t)row * ldc + q * 8) = cv[it];
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
  nxt.stores = nxt.pref ? Cfg::WTM / 8 : 0;
  return nxt;
}

// One 512-thread workgroup per CU walks its planned list (TileDesc table [k][gridDim.x], ended by the
// first empty slot). Tiles of the other bodies (w4a4 g128, E4M3, weight-only) run gg_v2_kernel's
// bodies with their own prologue and never take a prefetch.
template <int QM, int TRACE = 0, int SAUX = 16, int FILLALL = 0>
__global__ __launch_bounds__(512, 2) void gg_v2q_kernel(GGArgs args) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
  const int G = gridDim.x;
  QState st{false, 0, 0};
  for (int k = 0;; ++k) {
    const int idx = k * G + blockIdx.x;
    const TileDesc td = p_tile(args, idx);
    const int prob = uni(td.prob);
    if (prob < 0) break;
    const int nx_idx = uni(p_tile(args, idx + G).prob) >= 0 ? idx + G : -1;
    const int qt = uni(p_qtype(args, prob)), cls = uni(td.cls) & 0xFF;
    if (!st.pref && k > 0) {  // the previous tile's LDS use (split-K flag, other bodies) is over
      wait_vmcnt<0>();
      __syncthreads();
    }
    bool done = false;
#define MXMOE_V2Q(Q, BMC)                                                                                        \
  if (!done && (QM & (1 << Q)) && qt == Q && cls == BMC) {                                                       \
    st = gg_tile_v2q<V2Cfg<(BMC) == 0 ? 256 : (BMC) == 1 ? 128 : 64>, Q, TRACE, SAUX, FILLALL>(args, idx, nx_idx, st, lds); \
    done = true;                                                                                                 \
  }
    MXMOE_V2Q(QT_I8, 0)
    MXMOE_V2Q(QT_I8, 1)
    MXMOE_V2Q(QT_I4, 0)
    MXMOE_V2Q(QT_I4, 1)
    MXMOE_V2Q(QT_F16, 0)
    MXMOE_V2Q(QT_F16, 1)
    MXMOE_V2Q(QT_F16, 2)
    MXMOE_V2Q(QT_BF16, 0)
    MXMOE_V2Q(QT_BF16, 1)
    MXMOE_V2Q(QT_BF16, 2)
#undef MXMOE_V2Q
    if (!done) {  // the other tile bodies (their own prologue / LDS use)
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
      wait_vmcnt<0>();
      __syncthreads();  // the body's LDS use ends for every wave before the next tile's DMA
      st = QState{false, 0, 0};
    }
  }
}

}  // namespace mxmoe
