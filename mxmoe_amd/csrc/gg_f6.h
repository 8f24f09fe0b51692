// gg_f6.h — w4a4 tiles on the block-scaled fp6 MFMA (QT_I4F6). Included by gg_api.hip after
// gg_device.h.
//
// Reference path replaced: the w4a4_g-1_sym tile of the reference GroupGEMM (int4 x int4 MMA with
// an exact int32 accumulate, mm_tile.cuh:469-496 / cta_gemm.cuh:599-607 epilogue). gfx950 has no
// int4 MFMA; the int8 MFMA route (v3 / v2x) widens every nibble in registers (3 VALU per int4
// dword) and runs at the int8 rate. Here each int4 code v in [-8, 7] is re-encoded once, outside
// the GEMM, as an OCP FP6 E3M2 code (exact: E3M2 holds every integer of magnitude <= 8) and the
// tile runs v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales: the fp6 rate (~2x int8 on
// MI355X, tools/probe_f6.hip: 7.8 vs 4.3 POPS) and no widening VALU. The products are small
// integers and every f32 partial sum is an integer below 2^24 (|sum| <= 64 K, K <= 131072), so the
// f32 accumulator holds exactly the reference's int32 sum, whatever the summation order; the
// epilogue then rounds exactly as the int4 path (scale_pack4f on that value).
//
// fp6 image of a packed int4 row (mxmoe_gg_pack_f6): per K-128 block b, 96 bytes at 96 b:
//   bytes [0, 64): P, 16 B per lane group g (g < 4) = dwords 0-3 of group g's 32 codes
//   bytes [64, 96): Q, 8 B per group = dwords 4-5
// group g holds the 32 codes of int4 elements 128 b + 32 g + j (j < 32) in pack_wxax nibble order
// (element e = low nibble of byte e / 2 first), code j at bits [6 j, 6 j + 6) of the 192-bit value;
// elements past K are code 0. A and B use the same element order, so the MFMA's K sum is the
// reference's dot product (the sum is order-free). The MFMA lane map (checked by the probe on
// integer data): lane l holds row l & 15, codes of group l >> 4 of the K-128 step.
//
// LDS stage (K-128 of every tile row): A-P | A-Q | B-P | B-Q.
//   P images: 64-B rows, 16-B chunk c of row r at chunk c ^ swz64(r) (v3's image: the 16-row
//     ds_read_b128 of a fragment is conflict-free); filled by 16-row x 64-B buffer-form LDS-DMA
//   Q images: per 16-row fragment 512 B, group pair c = g >> 1 of row r at (16 c + r) * 16, so a
//     fragment's ds_read_b64 covers 256 contiguous bytes per half wave (conflict-free); filled by
//     half-wave (lanes 0-31) 16-B LDS-DMA pieces, one per 16-row fragment
// Ring of NBUF stages, DIST in flight (as v3: stage s + DIST is written into the buffer stage s - 1
// was read from, after the barrier that follows every wave's compute(s - 1)).
#pragma once

namespace mxmoe {

template <int BM_, int BN_ = 256, int WM_ = 2, int WN_ = 4, int NBUF_ = 3, int DIST_ = 2>
struct F6Cfg {
  static constexpr int BM = BM_, BN = BN_, NBUF = NBUF_, DIST = DIST_;
  static constexpr int WM = WM_, WN = WN_, NWAVES = WM * WN, NT = NWAVES * 64;
  static constexpr int SKB = 96;  // image bytes of one row per K-128 stage
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int AQ_OFF = BM * 64, BP_OFF = BM * 96, BQ_OFF = BM * 96 + BN * 64;
  static constexpr int STAGE_BYTES = (BM + BN) * SKB;
  // LDS-DMA pieces per wave per stage: P (16 rows x 64 B) and Q (16 rows x 32 B, half wave) per
  // 16-row fragment of A and of B
  static constexpr int GA = BM / (16 * NWAVES), GB = BN / (16 * NWAVES);
  static constexpr int DPS = 2 * (GA + GB);
  static constexpr int EPI_BYTES = WM * WN * WTM * WTN * 2;
  static constexpr int RING_BYTES = NBUF * STAGE_BYTES;
  static constexpr int LDS_BYTES = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
  static_assert(WTN == 64 || WTN == 128, "epilogue_v3 stages 128-B or 256-B rows");
  static_assert(GA >= 1 && GB >= 1 && GA * 16 * NWAVES == BM && GB * 16 * NWAVES == BN, "whole fragments per wave");
  static_assert(DIST < NBUF, "ring: stage s+DIST reuses the buffer of stage s-1 at most");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// fp6 x fp6 over K = 128, E3M2 codes (format 3) for both operands, block scales 2^0 (e8m0 127)
__device__ __forceinline__ v4f mfma_f6_k128(const v8i& b, const v8i& a, const v4f& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, 3, 3, 0, 127, 0, 127);
}

// OPT (lab A/B): 1 = fragment reads kept unpaired (no ds_read2st64_b64 of two Q fragments);
// 2 = the next stage's LDS-DMA spread through the MFMA stream (sched_group_barrier, as v3x)
template <class Cfg, int OPT = 0>
__device__ __forceinline__ void gg_tile_f6(const GGMeta& mt, const uint8_t* __restrict__ A,
                                           const uint8_t* __restrict__ B, const _Float16* __restrict__ SA,
                                           const _Float16* __restrict__ SB, _Float16* __restrict__ C, int m0, int n0,
                                           uint8_t* lds) {
  constexpr int FM = Cfg::FM, FN = Cfg::FN, GA = Cfg::GA, GB = Cfg::GB, DPS = Cfg::DPS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int r16 = lane & 15, g = lane >> 4;
  const int M = mt.M, N = mt.N;
  const int64_t lda = mt.lda_b, ldb = mt.ldb_b;
  const int nst = mt.kbytes / Cfg::SKB;  // the host pads image rows to whole K-128 stages

  // buffer-form LDS-DMA: per-tile resources, fixed 32-bit lane offsets, the stage in soffset
  const __amdgpu_buffer_rsrc_t rsA = v3_rsrc(A + (int64_t)m0 * lda);
  const __amdgpu_buffer_rsrc_t rsB = v3_rsrc(B + (int64_t)n0 * ldb);
  uint32_t voAP[GA], voAQ[GA], voBP[GB], voBQ[GB];
  {
    const int rsub = lane >> 2, p = lane & 3;  // P piece: lane -> row rsub, physical chunk p
    const int qc = (lane >> 4) & 1;            // Q piece (lanes 0-31): row r16, group pair qc
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int f0 = (wave * GA + j) * 16;
      const int rp = f0 + rsub, rq = f0 + r16;
      voAP[j] = (uint32_t)((min(m0 + rp, M - 1) - m0) * lda) + (uint32_t)((p ^ swz64(rp)) << 4);
      voAQ[j] = (uint32_t)((min(m0 + rq, M - 1) - m0) * lda) + 64u + (uint32_t)(qc << 4);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int f0 = (wave * GB + j) * 16;
      const int rp = f0 + rsub, rq = f0 + r16;
      voBP[j] = (uint32_t)((min(n0 + rp, N - 1) - n0) * ldb) + (uint32_t)((p ^ swz64(rp)) << 4);
      voBQ[j] = (uint32_t)((min(n0 + rq, N - 1) - n0) * ldb) + 64u + (uint32_t)(qc << 4);
    }
  }
  auto issue = [&](int s) {
    uint8_t* st = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES;
    const int so = s * Cfg::SKB;
#pragma unroll
    for (int j = 0; j < GA; ++j) v3_bdma(rsA, st + (wave * GA + j) * 1024, voAP[j], so);
#pragma unroll
    for (int j = 0; j < GB; ++j) v3_bdma(rsB, st + Cfg::BP_OFF + (wave * GB + j) * 1024, voBP[j], so);
    if (lane < 32) {
#pragma unroll
      for (int j = 0; j < GA; ++j) v3_bdma(rsA, st + Cfg::AQ_OFF + (wave * GA + j) * 512, voAQ[j], so);
#pragma unroll
      for (int j = 0; j < GB; ++j) v3_bdma(rsB, st + Cfg::BQ_OFF + (wave * GB + j) * 512, voBQ[j], so);
    }
  };

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0, 0, 0, 0};

  const uint32_t offP = (uint32_t)(((g ^ swz64(r16)) << 4) + r16 * 64);
  const uint32_t offQ = (uint32_t)((((g >> 1) * 16 + r16) << 4) + (g & 1) * 8);
  auto frag = [&](const uint8_t* P, const uint8_t* Q) {
    const v4i p = *reinterpret_cast<const v4i*>(P + offP);
    const v2i q = *reinterpret_cast<const v2i*>(Q + offQ);
    if constexpr ((OPT & 1) != 0) asm volatile("");
    return v8i{p[0], p[1], p[2], p[3], q[0], q[1], 0, 0};
  };
  auto compute = [&](int s) {
    const uint8_t* st = lds + (s % Cfg::NBUF) * Cfg::STAGE_BYTES;
    const uint8_t* AP = st + wm * Cfg::WTM * 64;
    const uint8_t* AQ = st + Cfg::AQ_OFF + wm * Cfg::WTM * 32;
    const uint8_t* BP = st + Cfg::BP_OFF + wn * Cfg::WTN * 64;
    const uint8_t* BQ = st + Cfg::BQ_OFF + wn * Cfg::WTN * 32;
    v8i b[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = frag(BP + j * 1024, BQ + j * 512);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const v8i a = frag(AP + i * 1024, AQ + i * 512);
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma_f6_k128(b[j], a, acc[i][j]);
    }
  };

#pragma unroll
  for (int p = 0; p < Cfg::DIST; ++p)
    if (p < nst) issue(p);
  for (int s = 0; s < nst; ++s) {
    const int later = min(Cfg::DIST - 1, nst - 1 - s);  // stages issued after s so far
    if (later >= 2) wait_vmcnt<2 * DPS>();
    else if (later == 1) wait_vmcnt<DPS>();
    else wait_vmcnt<0>();
    lds_barrier();  // stage s landed for every wave; every wave is done with buffer (s-1) % NBUF
    if (s + Cfg::DIST < nst) issue(s + Cfg::DIST);
    compute(s);
    if constexpr ((OPT & 2) != 0) {
      constexpr int KS = FM * FN / DPS > 0 ? FM * FN / DPS : 1;
#pragma unroll
      for (int q = 0; q < DPS; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);  // KS MFMAs
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // one VMEM read (LDS-DMA)
      }
    }
  }
  wait_vmcnt<0>();
  lds_barrier();  // ring -> epilogue staging
  epilogue_v3<Cfg, QT_I4F6>(mt, acc, SA, SB, C, m0, n0, lds);
}

// One 512-thread workgroup per CU (2 waves per SIMD: <= 256 VGPRs); 256-row tiles and the
// 128-row tail class (TileDesc::cls 1). Planned for QT_I4F6 problems only.
template <int NBUF, int DIST, int OPT = 0>
__global__ __launch_bounds__(512, 2) void gg_f6_kernel(GGArgs args) {
  typedef F6Cfg<256, 256, 2, 4, NBUF, DIST> CT;
  typedef F6Cfg<128, 256, 2, 4, NBUF, DIST> CS;
  __shared__ __attribute__((aligned(16))) uint8_t lds[CT::LDS_BYTES];
  const TileDesc td = args.tiles[blockIdx.x];
  if (td.prob < 0) return;
  const GGMeta mt = args.meta[td.prob];
  if (mt.qtype != QT_I4F6) return;  // (the planner never places another type on this kernel)
  const uint8_t* A = static_cast<const uint8_t*>(args.ptr_A[td.prob]);
  const uint8_t* B = static_cast<const uint8_t*>(args.ptr_B[td.prob]);
  const _Float16* SA = static_cast<const _Float16*>(args.ptr_SA[td.prob]);
  const _Float16* SB = static_cast<const _Float16*>(args.ptr_SB[td.prob]);
  _Float16* C = static_cast<_Float16*>(args.ptr_C[td.prob]);
  if (td.cls == 0) gg_tile_f6<CT, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
  else gg_tile_f6<CS, OPT>(mt, A, B, SA, SB, C, td.m0, td.n0, lds);
}

// ---- int4 (pack_wxax rows) -> fp6 image (mxmoe_gg_pack_f6) ----
// e3m2 code of each int4 nibble n (two's complement): bytes n = 0..7 and n = 8..15
constexpr uint64_t kF6LutLo = 0x1716151412100C00ull;  // 0, 1, 2, 3, 4, 5, 6, 7
constexpr uint64_t kF6LutHi = 0x2C30323435363738ull;  // -8, -7, -6, -5, -4, -3, -2, -1

__host__ __device__ inline uint32_t f6_code(uint32_t nib) {
  return (uint32_t)(((nib < 8 ? kF6LutLo : kF6LutHi) >> (8 * (nib & 7))) & 63u);
}

// 32 nibbles (w[0..3], element j = nibble j & 7 of dword j >> 3) -> 6 dwords, code j at bit 6 j
__host__ __device__ inline void f6_pack32(const uint32_t w[4], uint32_t d[6]) {
  for (int i = 0; i < 6; ++i) d[i] = 0;
  for (int j = 0; j < 32; ++j) {
    const uint32_t c = f6_code((w[j >> 3] >> (4 * (j & 7))) & 15u);
    const int bit = 6 * j, o = bit & 31;
    d[bit >> 5] |= c << o;
    if (o > 26) d[(bit >> 5) + 1] |= c >> (32 - o);
  }
}

// one thread per (row, K-128 block, lane group): 16 source bytes -> 16 B of P + 8 B of Q
__global__ __launch_bounds__(256) void f6_pack_kernel(const uint8_t* __restrict__ src, int64_t ld_src,
                                                      uint8_t* __restrict__ dst, int64_t ld_dst, int rows, int K) {
  const int nblk = (K + 127) / 128;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)rows * nblk * 4) return;
  const int g = (int)(t & 3);
  const int64_t rb = t >> 2;
  const int b = (int)(rb % nblk);
  const int64_t row = rb / nblk;
  const int e0 = b * 128 + g * 32;  // first element of the group
  uint32_t w[4] = {0, 0, 0, 0};
  const uint8_t* s = src + row * ld_src + e0 / 2;
  if (e0 + 32 <= K) {
    const uint4 v = *reinterpret_cast<const uint4*>(s);
    w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
  } else {
    for (int e = e0; e < K; e += 2) w[(e - e0) >> 3] |= (uint32_t)s[(e - e0) >> 1] << (4 * ((e - e0) & 7));
  }
  uint32_t d[6];
  f6_pack32(w, d);
  uint8_t* o = dst + row * ld_dst + b * 96;
  *reinterpret_cast<uint4*>(o + g * 16) = uint4{d[0], d[1], d[2], d[3]};
  *reinterpret_cast<uint2*>(o + 64 + g * 8) = uint2{d[4], d[5]};
}

}  // namespace mxmoe
