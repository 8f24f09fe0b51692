// moe_ops.hip — MoE-layer plumbing around the GroupGEMM (include/mxmoe_moe.h), gfx950.
//
// Reference (SeaCatComplexes/MxMoE, mxmoe/kernels/src/ref_bind.cu; read as text only):
//   gg_permute_inp: sort(topk_ids) / floor_divide(topk) / bincount ......... ref_bind.cu:47-64, 452-456
//   quant_inp_act -> quant_act_kernel (per-expert activation quantisation) .. :434-592
//   silu_mul_then_quant -> silu_mul_then_quant_kernel ....................... :595-757
//   gg_unpermute_out (empty stub) ........................................... :66
// The reference's device kernels (act_kernel.cuh) are absent from its tree; the quantiser here is
// its quant_weight (quantize.cuh:218-279) per token row / 128-element group + pack_wxax
// (quantize.cuh:425-475), i.e. exactly the operand format of the GroupGEMM.
//
// All four kernels are HBM-bound byte movers: one workgroup per row (token or slot), 16-B
// coalesced loads of 8 fp16 per lane, reductions in registers / lane shuffles, stores of the packed
// codes as one 4-B (int4) / 8-B (int8) / 16-B (fp16) word per lane — no LDS tiling, no MFMA.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/mxmoe_gg.h"
#include "../../include/mxmoe_moe.h"

namespace mxmoe {
namespace detail {
int set_error(int code, const std::string& msg);  // gg_api.hip (thread-local mxmoe_gg_last_error)
}

namespace {

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return detail::set_error(code, buf);
}

constexpr int kThreads = 256;
constexpr int kRouteThreads = 1024;
constexpr int kChunk = kThreads * 8;     // fp16 elements one pass of the workgroup covers
constexpr int kMaxChunks = 8;            // rows up to 16384 elements
constexpr int kMaxWidth = kChunk * kMaxChunks;

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int wave_incl_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// exclusive block prefix of v (NT threads) and the block total
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* total, int* lds4) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int incl = wave_incl_scan(v);
  if (lane == 63) lds4[wave] = incl;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    base += w < wave ? lds4[w] : 0;
    tot += lds4[w];
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// ---------------------------------------------------------------------------------------------
// route: workgroup e finds every id == e in flattened order (stable), its slot base = #ids < e.
// Each thread scans a contiguous run of the ids twice (count, then place); the runs' counts are
// prefix-summed across the workgroup so the placement keeps the flattened order.
__global__ __launch_bounds__(kRouteThreads) void route_kernel(const int32_t* __restrict__ ids, int n, int topk,
                                                              int32_t* __restrict__ sorted, int32_t* __restrict__ perm,
                                                              int32_t* __restrict__ inv, int32_t* __restrict__ counts) {
  __shared__ int lds[kRouteThreads / 64];
  const int e = blockIdx.x;
  // run of 4*q ids per thread (q int4 words, read as independent 16-B loads); ids past n read as -1
  const int q = (n + 4 * kRouteThreads - 1) / (4 * kRouteThreads);
  const int b = threadIdx.x * q * 4;
  auto id4 = [&](int w) -> int4 {
    const int i = b + 4 * w;
    if (i + 4 <= n && (n & 3) == 0) return *reinterpret_cast<const int4*>(ids + i);
    int4 v;
    v.x = i < n ? ids[i] : -1;
    v.y = i + 1 < n ? ids[i + 1] : -1;
    v.z = i + 2 < n ? ids[i + 2] : -1;
    v.w = i + 3 < n ? ids[i + 3] : -1;
    return v;
  };
  int less = 0, eq = 0;
#pragma unroll 8
  for (int w = 0; w < q; ++w) {
    const int4 v = id4(w);
    less += (v.x >= 0 && v.x < e) + (v.y >= 0 && v.y < e) + (v.z >= 0 && v.z < e) + (v.w >= 0 && v.w < e);
    eq += (v.x == e) + (v.y == e) + (v.z == e) + (v.w == e);
  }
  int eq_total, less_total;
  const int rank = block_excl_scan<kRouteThreads>(eq, &eq_total, lds);
  block_excl_scan<kRouteThreads>(less, &less_total, lds);
  if (threadIdx.x == 0) counts[e] = eq_total;
  if (eq == 0) return;
  int pos = less_total + rank;
  for (int w = 0; w < q && eq > 0; ++w) {
    const int4 v = id4(w);
    const int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (vv[j] == e) {
        const int i = b + 4 * w + j;
        sorted[pos] = e;
        perm[pos] = i / topk;
        inv[i] = pos;
        ++pos;
        --eq;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
struct ActArgs {
  const _Float16* src;         // quant: hidden [T][K]; silu: routed gate_up [T*topk][2N]
  const _Float16* src_shared;  // silu: shared gate_up [T][2Ns] (quant: = src)
  int64_t ntk;                 // T * topk routed slots
  int64_t nslots;              // end of the launch's slot range (ntk, + T shared slots)
  int64_t s0;                  // first slot of the launch
  int K;                       // quant: row width of hidden
  int N, Ns;                   // silu: routed / shared intermediate width
  const int32_t* sorted;
  const int32_t* perm;
  const mxmoe_moe_seg* segs;
  int nseg;
  uint8_t* out;
  _Float16* scales;
  int64_t blk_shared;          // parts > 1: first workgroup of the shared rows (one row per workgroup)
  int parts;                   // 1, or 4: a shared row is split over the 4 waves of its workgroup
};

// quant_weight arithmetic (quantize.cuh:218-279): scale = fp16(amax / qmax), 0 -> 1;
// q = rint_even(clamp(fp16(x / scale), -qmax, qmax))
__device__ __forceinline__ _Float16 rtn_scale(float amax, float qmax) {
  _Float16 s = (_Float16)(amax / qmax);
  return s == (_Float16)0 ? (_Float16)1 : s;
}
// fp16(f32(x) / f32(s)) without the IEEE divide sequence (~10 VALU, which made these kernels
// VALU-bound): q = x * r, one Newton step q' = q + (x - q s) r with r = v_rcp_f32(s) (<= 1 ulp).
// q' is within 0.5 ulp (+ 2^-46 relative) of x / s. For fp16 x and s (11-bit significands) x / s is
// at least 1 / ((2^11 - 1)(2^12 - 1)) > 2^-23 (relative) away from every fp16 rounding midpoint
// (a 12-bit odd significand M with |x - M s| > 0 is at least one unit of the 23-bit product M s),
// so q' and the correctly rounded quotient lie on the same side of every midpoint and round to the
// same fp16 — bit-exact with the IEEE division the oracle uses.
__device__ __forceinline__ float div_f16_operands(float x, float s, float r) {
  const float q = x * r;
  return fmaf(fmaf(-q, s, x), r, q);
}
typedef _Float16 h2_t __attribute__((ext_vector_type(2)));

// Codes of elements 2p, 2p+1 of x: d = fp16(x / s) clamped to +-qmax in fp16 (exact), then
// d + 1536 in fp16: for |d| <= 127 the sum lies in [1024, 2048) where the fp16 spacing is 1, so
// the add rounds d to an integer with ties to even (1536 is even: rint's tie rule), and the low
// byte of the sum's bits (mantissa 512 + rint(d)) is rint(d)'s two's-complement byte. Returns the
// pair's bits: code(2p) in byte 0, code(2p+1) in byte 2.
__device__ __forceinline__ uint32_t pair_codes(const h8_t& x, int p, float s, float r, h2_t lim) {
  h2_t d = {(_Float16)div_f16_operands((float)x[2 * p], s, r), (_Float16)div_f16_operands((float)x[2 * p + 1], s, r)};
  d = __builtin_elementwise_min(__builtin_elementwise_max(d, -lim), lim);
  d = d + h2_t{(_Float16)1536, (_Float16)1536};
  return __builtin_bit_cast(uint32_t, d);
}
// pack_wxax (quantize.cuh:425-475) stores element j+x of a 16-bit word at bits (PACK-1-x)*bits:
// int8 word j = q[2j] << 8 | q[2j+1] (little-endian bytes q[2j+1], q[2j]); int4 word j =
// q[4j] << 12 | q[4j+1] << 8 | q[4j+2] << 4 | q[4j+3].
// order4: 4 codes from two pair words as bytes [q1, q0, q3, q2] (v_perm_b32: selectors 0-3 take
// the second operand's bytes, 4-7 the first's)
__device__ __forceinline__ uint32_t order4(uint32_t p01, uint32_t p23) { return __builtin_amdgcn_perm(p23, p01, 0x04060002u); }
// int8: 8 codes -> 8 packed bytes
__device__ __forceinline__ uint2 codes_i8(const h8_t& x, float s, float r, h2_t lim) {
  return uint2{order4(pair_codes(x, 0, s, r, lim), pair_codes(x, 1, s, r, lim)),
               order4(pair_codes(x, 2, s, r, lim), pair_codes(x, 3, s, r, lim))};
}
// int4: from [q1, q0, q3, q2] nibbles, t = a | a >> 4 puts (q0 << 4 | q1) in byte 0 and
// (q2 << 4 | q3) in byte 2; the word is bytes [t.2, t.0, u.2, u.0] (pack_i4x8 order)
__device__ __forceinline__ uint32_t codes_i4(const h8_t& x, float s, float r, h2_t lim) {
  const uint32_t a = order4(pair_codes(x, 0, s, r, lim), pair_codes(x, 1, s, r, lim)) & 0x0F0F0F0Fu;
  const uint32_t b = order4(pair_codes(x, 2, s, r, lim), pair_codes(x, 3, s, r, lim)) & 0x0F0F0F0Fu;
  return __builtin_amdgcn_perm(b | (b >> 4), a | (a >> 4), 0x04060002u);
}
// max |x| over 8 fp16 (exact in fp16: v_pk_max_f16 on sign-cleared pairs)
__device__ __forceinline__ float amax8(const h8_t& x) {
  const uint4 w = __builtin_bit_cast(uint4, x);
  const uint32_t m = 0x7FFF7FFFu;
  const h2_t a = __builtin_elementwise_max(__builtin_bit_cast(h2_t, w.x & m), __builtin_bit_cast(h2_t, w.y & m));
  const h2_t b = __builtin_elementwise_max(__builtin_bit_cast(h2_t, w.z & m), __builtin_bit_cast(h2_t, w.w & m));
  const h2_t c = __builtin_elementwise_max(a, b);
  return fmaxf((float)c[0], (float)c[1]);
}

// One WAVE per slot row (4 rows per 256-thread workgroup): lane l holds elements c*512 + 8l .. +7
// of chunk c in registers (MAXC chunks: rows up to MAXC*512 elements, MAXC = the launch's widest
// row in 512-element chunks), so every lane has MAXC independent 16-B loads in flight, the
// per-token amax is a wave butterfly and a 128-element group is 16 adjacent lanes — no LDS, no
// barrier. Loads and the SiLU are straight-line over all MAXC chunks (lanes past the row read the
// row's first 16 B and zero them by a select): per-chunk branches kept the scheduler from
// interleaving the chunks' dependency chains (v_exp / v_rcp latency, packed-math wait states). parts == 4: the workgroups from blk_shared on take one
// wide shared row each, wave w its w-th run of 128-aligned columns (the per-token amax then crosses
// the 4 waves through LDS), so routed and shared rows share one launch and one register budget.
// MODE 0: quant_act (routed slot s gathers hidden[perm[s]], width K); 1: silu_mul_quant (slot rows
// [gate | up] of the gate_up output); 2: quant_slots (slot rows already activated: the gate_up
// GroupGEMM's fused SiLU epilogue, routed [T*topk][N], shared [T][Ns]); 3: silu_mul_quant on a
// gate_up output whose gate / up columns alternate in 16-column blocks (the interleaved weights of
// the fused epilogue, run through the plain epilogue: small-batch calls on wo3)
template <int MODE, int MAXC>
__global__ __launch_bounds__(kThreads) void act_quant_kernel(ActArgs a) {
  constexpr bool SILU = MODE == 1 || MODE == 3;
  __shared__ float wave_amax[kThreads / 64];
  const int lane = threadIdx.x & 63;
  const bool split_row = a.parts > 1 && (int64_t)blockIdx.x >= a.blk_shared;  // workgroup-uniform
  const int part = split_row ? (int)(threadIdx.x >> 6) : 0;
  const int64_t s = split_row ? a.ntk + ((int64_t)blockIdx.x - a.blk_shared)
                              : a.s0 + (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (s >= (a.parts > 1 && !split_row ? a.ntk : a.nslots)) return;  // split_row: uniform
  int e;
  const _Float16* row_src;
  if (s < a.ntk) {
    e = a.sorted[s];
    row_src = (MODE == 1 || MODE == 3) ? a.src + s * 2 * (int64_t)a.N
            : MODE == 2 ? a.src + s * (int64_t)a.N
                        : a.src + (int64_t)a.perm[s] * a.K;
  } else {
    e = a.nseg - 1;
    const int64_t t = s - a.ntk;
    row_src = (MODE == 1 || MODE == 3) ? a.src_shared + t * 2 * (int64_t)a.Ns
            : MODE == 2 ? a.src_shared + t * (int64_t)a.Ns
                        : a.src + t * a.K;
  }
  if (e < 0 || e >= a.nseg) return;  // invalid id: the slot was never routed (route ignores it)
  const mxmoe_moe_seg sg = a.segs[e];
  const int64_t row = s - sg.first_slot;
  if (row < 0 || row >= sg.rows) return;  // slot outside its segment (inconsistent table): never write
  const int upoff = SILU ? (s < a.ntk ? a.N : a.Ns) : 0;  // column of the "up" half
  // this wave's columns [col0, col0 + width) of the row (split rows: 128-aligned quarter runs)
  const int qw = split_row ? ((sg.width / 4 + 127) & ~127) : sg.width;
  const int col0 = part * qw;
  const int width = split_row ? max(0, min(qw, sg.width - col0)) : sg.width;
  // (a wave whose quarter of a split row is empty keeps a valid address: the row's start)
  const _Float16* const base = width > 0 ? row_src + (MODE == 3 ? 2 * col0 : col0) : row_src;

  // every load of the row first (all in flight together), then the arithmetic
  h8_t x[MAXC];
  h8_t u[SILU ? MAXC : 1];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int idx = c * 512 + lane * 8;
    const bool in = idx < width;
    const int li = in ? idx : 0;
    // (MODE 3: element e of the row sits at 2 (e & ~15) + (e & 15), its up value 16 further)
    const int gi = MODE == 3 ? 2 * (li & ~15) + (li & 15) : li;
    const uint4 xv = *reinterpret_cast<const uint4*>(base + gi);
    const uint4 z = {0, 0, 0, 0};
    x[c] = __builtin_bit_cast(h8_t, in ? xv : z);
    if constexpr (SILU) {
      const uint4 uv = *reinterpret_cast<const uint4*>(base + (MODE == 3 ? gi + 16 : upoff + li));
      u[c] = __builtin_bit_cast(h8_t, in ? uv : z);
    }
  }
  if constexpr (SILU) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {  // (zeros past the row: silu(0) * 0 = 0)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // silu(g) = g / (1 + e^-g) with the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: the
        // reference kernel is absent, so this is our definition; oracle/moe_ref.py allows 1 ulp)
        const float g = (float)x[c][j];
        const float sg = g * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g * -1.4426950408889634f));
        x[c][j] = (_Float16)(sg * (float)u[c][j]);
      }
    }
  }

  if (sg.qtag == MXMOE_ACT_FP16) {
    _Float16* o = reinterpret_cast<_Float16*>(a.out + sg.out_off) + row * sg.width + col0;  // (width 0: no store)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int idx = c * 512 + lane * 8;
      if (idx < width) *reinterpret_cast<h8_t*>(o + idx) = x[c];
    }
    return;
  }
  const int bits = sg.qtag == MXMOE_ACT_INT8 ? 8 : 4;
  const float qmax = bits == 8 ? 127.0f : 7.0f;
  const h2_t lim = {(_Float16)qmax, (_Float16)qmax};
  uint8_t* o = a.out + sg.out_off + (row * (int64_t)sg.width + col0) * bits / 8;
  if (sg.qtag == MXMOE_ACT_INT4_G128) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c * 512 >= width) break;  // uniform
      const int idx = c * 512 + lane * 8;
      float m = amax8(x[c]);
#pragma unroll
      for (int d = 8; d >= 1; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
      if (idx < width) {
        const _Float16 sc = rtn_scale(m, qmax);
        const float rs = __builtin_amdgcn_rcpf((float)sc);
        *reinterpret_cast<uint32_t*>(o + idx / 2) = codes_i4(x[c], (float)sc, rs, lim);
        if ((lane & 15) == 0) a.scales[sg.scale_off + (int64_t)((col0 + idx) / 128) * sg.rows + row] = sc;
      }
    }
    return;
  }
  float m = 0.0f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) m = fmaxf(m, amax8(x[c]));  // chunks past the row are zeros
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = fmaxf(m, __shfl_xor(m, d, 64));
  if (split_row) {  // every wave of the workgroup reaches here (its row's checks are uniform)
    if (lane == 0) wave_amax[part] = m;
    __syncthreads();
    m = fmaxf(fmaxf(wave_amax[0], wave_amax[1]), fmaxf(wave_amax[2], wave_amax[3]));
  }
  const _Float16 sc = rtn_scale(m, qmax);
  const float rs = __builtin_amdgcn_rcpf((float)sc);
  if (lane == 0 && part == 0) a.scales[sg.scale_off + row] = sc;
  // every chunk's codes first (straight-line: the chunks' packed-math chains interleave), then the
  // predicated stores
  if (bits == 8) {
    uint2 q[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) q[c] = codes_i8(x[c], (float)sc, rs, lim);
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c * 512 + lane * 8 < width) *reinterpret_cast<uint2*>(o + c * 512 + lane * 8) = q[c];
  } else {
    uint32_t q[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) q[c] = codes_i4(x[c], (float)sc, rs, lim);
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c * 512 + lane * 8 < width) *reinterpret_cast<uint32_t*>(o + (c * 512 + lane * 8) / 2) = q[c];
  }
}

// ---------------------------------------------------------------------------------------------
// combine: one workgroup per token, 8 fp16 columns per lane and pass
__global__ __launch_bounds__(kThreads) void combine_kernel(const _Float16* __restrict__ y, const int32_t* __restrict__ inv,
                                                           const float* __restrict__ w, const _Float16* __restrict__ shared,
                                                           const float* __restrict__ shared_w, int topk, int H,
                                                           _Float16* __restrict__ out) {
  const int64_t t = blockIdx.x;
  for (int idx = threadIdx.x * 8; idx < H; idx += kChunk) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < topk; ++k) {
      const int64_t slot = inv[t * topk + k];
      const float wk = w[t * topk + k];
      const h8_t v = *reinterpret_cast<const h8_t*>(y + slot * H + idx);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(wk, (float)v[j], acc[j]);
    }
    if (shared) {
      const float ws = shared_w ? shared_w[t] : 1.0f;
      const h8_t v = *reinterpret_cast<const h8_t*>(shared + t * H + idx);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(ws, (float)v[j], acc[j]);
    }
    h8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (_Float16)acc[j];
    *reinterpret_cast<h8_t*>(out + t * H + idx) = r;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace
}  // namespace mxmoe

using namespace mxmoe;

// registers sized to the widest row of the launch, in 512-element chunks (1408 -> 3, 2048 -> 4)
template <int MODE>
static void launch_act_w(const ActArgs& a, int maxw, hipStream_t st) {
  const int64_t blocks = a.parts > 1 ? a.blk_shared + (a.nslots - a.ntk)
                                     : (a.nslots - a.s0 + kThreads / 64 - 1) / (kThreads / 64);
  const dim3 grid((unsigned)blocks), block(kThreads);
  const int nc = (maxw + 511) / 512;
  if (nc <= 1) hipLaunchKernelGGL((act_quant_kernel<MODE, 1>), grid, block, 0, st, a);
  else if (nc <= 2) hipLaunchKernelGGL((act_quant_kernel<MODE, 2>), grid, block, 0, st, a);
  else if (nc <= 3) hipLaunchKernelGGL((act_quant_kernel<MODE, 3>), grid, block, 0, st, a);
  else if (nc <= 4) hipLaunchKernelGGL((act_quant_kernel<MODE, 4>), grid, block, 0, st, a);
  else if (nc <= 6) hipLaunchKernelGGL((act_quant_kernel<MODE, 6>), grid, block, 0, st, a);
  else if (nc <= 8) hipLaunchKernelGGL((act_quant_kernel<MODE, 8>), grid, block, 0, st, a);
  else if (nc <= 12) hipLaunchKernelGGL((act_quant_kernel<MODE, 12>), grid, block, 0, st, a);
  else if (nc <= 16) hipLaunchKernelGGL((act_quant_kernel<MODE, 16>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((act_quant_kernel<MODE, 32>), grid, block, 0, st, a);
}

// slots [0, nslots): one launch; rows of different widths (routed [0, ntk), shared [ntk, nslots)):
// one launch with each shared row split over a workgroup's 4 waves when a quarter of the shared row
// fits the routed rows' register width, else two launches, each with the register row of its width
template <int MODE>
static void launch_act_m(const ActArgs& a, int maxw, hipStream_t st) {
  launch_act_w<MODE>(a, maxw, st);
}
static void launch_act_any(int mode, const ActArgs& a, int maxw, hipStream_t st) {
  if (mode == 1) launch_act_m<1>(a, maxw, st);
  else if (mode == 2) launch_act_m<2>(a, maxw, st);
  else if (mode == 3) launch_act_m<3>(a, maxw, st);
  else launch_act_m<0>(a, maxw, st);
}
static int launch_act(int mode, ActArgs a, int64_t nslots, int w_routed, int w_shared, void* stream) {
  if (nslots == 0) return MXMOE_GG_OK;
  a.parts = 1;
  a.blk_shared = 0;
  const int qw = (w_shared / 4 + 127) & ~127;
  if (nslots > a.ntk && a.ntk > 0 && w_shared > w_routed && qw <= w_routed) {
    a.parts = 4;
    a.blk_shared = (a.ntk + kThreads / 64 - 1) / (kThreads / 64);
    a.s0 = 0;
    a.nslots = nslots;
    launch_act_any(mode, a, w_routed, (hipStream_t)stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MXMOE_GG_ERR_HIP, "act_quant_kernel launch failed: %s", hipGetErrorString(e));
    return MXMOE_GG_OK;
  }
  const bool split = nslots > a.ntk && w_routed != w_shared && a.ntk > 0;
  a.s0 = 0;
  a.nslots = split ? a.ntk : nslots;
  const int w0 = split ? w_routed : (nslots > a.ntk ? (w_routed > w_shared ? w_routed : w_shared) : w_routed);
  launch_act_any(mode, a, w0, (hipStream_t)stream);
  if (split) {
    a.s0 = a.ntk;
    a.nslots = nslots;
    launch_act_any(mode, a, w_shared, (hipStream_t)stream);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MXMOE_GG_ERR_HIP, "act_quant_kernel launch failed: %s", hipGetErrorString(e));
  return MXMOE_GG_OK;
}

extern "C" {

int mxmoe_moe_route(const int32_t* topk_ids, int64_t T, int topk, int E, int32_t* sorted_expert,
                    int32_t* perm_token, int32_t* inv_slot, int32_t* counts, void* stream) {
  if (T < 0 || topk <= 0 || E <= 0 || E > 4096 || T * topk > (int64_t)1 << 30)
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_route: bad sizes (T=%lld topk=%d E=%d)", (long long)T, topk, E);
  if (T > 0 && (!topk_ids || !sorted_expert || !perm_token || !inv_slot))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_route: NULL pointer");
  if (!counts) return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_route: NULL counts");
  hipLaunchKernelGGL(route_kernel, dim3(E), dim3(kRouteThreads), 0, (hipStream_t)stream, topk_ids, (int)(T * topk), topk,
                     sorted_expert, perm_token, inv_slot, counts);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MXMOE_GG_ERR_HIP, "route_kernel launch failed: %s", hipGetErrorString(e));
  return MXMOE_GG_OK;
}

int mxmoe_moe_quant_act(const void* hidden, int64_t T, int K, int topk, int with_shared,
                        const int32_t* sorted_expert, const int32_t* perm_token, const mxmoe_moe_seg* segs, int nseg,
                        void* out, void* scales, void* stream) {
  if (T < 0 || topk <= 0 || nseg <= 0 || K <= 0 || K % 128 || K > kMaxWidth)
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_quant_act: need K %% 128 == 0, K <= %d, topk > 0, nseg > 0 (K=%d)",
                kMaxWidth, K);
  if (T > 0 && (!hidden || !sorted_expert || !perm_token || !segs || !out || !aligned16(hidden) || !aligned16(out)))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_quant_act: NULL or misaligned pointer (hidden / out need 16 B)");
  const ActArgs a{static_cast<const _Float16*>(hidden), static_cast<const _Float16*>(hidden), T * topk, 0, 0, K, 0, 0,
                  sorted_expert, perm_token, segs, nseg, static_cast<uint8_t*>(out), static_cast<_Float16*>(scales)};
  return launch_act(0, a, T * topk + (with_shared ? T : 0), K, K, stream);
}

int mxmoe_moe_silu_mul_quant(const void* routed_in, const void* shared_in, int64_t T, int topk, int N, int N_shared,
                             const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg, void* out,
                             void* scales, void* stream) {
  if (T < 0 || topk <= 0 || nseg <= 0 || N <= 0 || N % 128 || N > kMaxWidth ||
      (shared_in && (N_shared <= 0 || N_shared % 128 || N_shared > kMaxWidth)))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_silu_mul_quant: widths must be multiples of 128 and <= %d (N=%d, "
                "N_shared=%d)", kMaxWidth, N, N_shared);
  if (T > 0 && (!routed_in || !sorted_expert || !segs || !out || !aligned16(routed_in) || !aligned16(out) ||
                (shared_in && !aligned16(shared_in))))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_silu_mul_quant: NULL or misaligned pointer (16 B)");
  const ActArgs a{static_cast<const _Float16*>(routed_in), static_cast<const _Float16*>(shared_in), T * topk, 0, 0, 0,
                  N, N_shared, sorted_expert, nullptr, segs, nseg, static_cast<uint8_t*>(out),
                  static_cast<_Float16*>(scales)};
  return launch_act(1, a, T * topk + (shared_in ? T : 0), N, shared_in ? N_shared : N, stream);
}

int mxmoe_moe_silu_mul_quant_il(const void* routed_in, const void* shared_in, int64_t T, int topk, int N,
                                int N_shared, const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg,
                                void* out, void* scales, void* stream) {
  if (T < 0 || topk <= 0 || nseg <= 0 || N <= 0 || N % 128 || N > kMaxWidth ||
      (shared_in && (N_shared <= 0 || N_shared % 128 || N_shared > kMaxWidth)))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_silu_mul_quant_il: widths must be multiples of 128 and <= %d (N=%d, "
                "N_shared=%d)", kMaxWidth, N, N_shared);
  if (T > 0 && (!routed_in || !sorted_expert || !segs || !out || !aligned16(routed_in) || !aligned16(out) ||
                (shared_in && !aligned16(shared_in))))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_silu_mul_quant_il: NULL or misaligned pointer (16 B)");
  const ActArgs a{static_cast<const _Float16*>(routed_in), static_cast<const _Float16*>(shared_in), T * topk, 0, 0, 0,
                  N, N_shared, sorted_expert, nullptr, segs, nseg, static_cast<uint8_t*>(out),
                  static_cast<_Float16*>(scales)};
  return launch_act(3, a, T * topk + (shared_in ? T : 0), N, shared_in ? N_shared : N, stream);
}

int mxmoe_moe_quant_slots(const void* routed_in, const void* shared_in, int64_t T, int topk, int N, int N_shared,
                          const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg, void* out, void* scales,
                          void* stream) {
  if (T < 0 || topk <= 0 || nseg <= 0 || N <= 0 || N % 128 || N > kMaxWidth ||
      (shared_in && (N_shared <= 0 || N_shared % 128 || N_shared > kMaxWidth)))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_quant_slots: widths must be multiples of 128 and <= %d (N=%d, "
                "N_shared=%d)", kMaxWidth, N, N_shared);
  if (T > 0 && (!routed_in || !sorted_expert || !segs || !out || !aligned16(routed_in) || !aligned16(out) ||
                (shared_in && !aligned16(shared_in))))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_quant_slots: NULL or misaligned pointer (16 B)");
  const ActArgs a{static_cast<const _Float16*>(routed_in), static_cast<const _Float16*>(shared_in), T * topk, 0, 0, 0,
                  N, N_shared, sorted_expert, nullptr, segs, nseg, static_cast<uint8_t*>(out),
                  static_cast<_Float16*>(scales)};
  return launch_act(2, a, T * topk + (shared_in ? T : 0), N, shared_in ? N_shared : N, stream);
}

int mxmoe_moe_combine(const void* y, const int32_t* inv_slot, const float* weights, const void* shared,
                      const float* shared_w, int64_t T, int topk, int H, void* out, void* stream) {
  if (T < 0 || topk <= 0 || H <= 0 || H % 8)
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_combine: need H %% 8 == 0, topk > 0 (H=%d)", H);
  if (T == 0) return MXMOE_GG_OK;
  if (!y || !inv_slot || !weights || !out || !aligned16(y) || !aligned16(out) || (shared && !aligned16(shared)))
    return fail(MXMOE_GG_ERR_INVALID, "mxmoe_moe_combine: NULL or misaligned pointer (16 B)");
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)T), dim3(kThreads), 0, (hipStream_t)stream,
                     static_cast<const _Float16*>(y), inv_slot, weights, static_cast<const _Float16*>(shared), shared_w,
                     topk, H, static_cast<_Float16*>(out));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(MXMOE_GG_ERR_HIP, "combine_kernel launch failed: %s", hipGetErrorString(e));
  return MXMOE_GG_OK;
}

}  // extern "C"
