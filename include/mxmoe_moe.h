/*
 * mxmoe_moe.h — C-ABI of the MoE-layer plumbing around the GroupGEMM (MI355X / gfx950):
 * token routing (permute), per-expert activation quantisation, SiLU·mul + quantisation of the
 * gate_up output, and the weighted combine (unpermute). SURVEY.md §8(f) rank 2.
 *
 * Reference interface each entry point replaces (SeaCatComplexes/MxMoE, mxmoe/kernels/src/ref_bind.cu,
 * the torch extension `mxmoe_ops`):
 *   mxmoe_moe_route ............ gg_permute_inp (ref_bind.cu:47-64) and the sort / bincount at the
 *                                head of quant_inp_act (:452-456): values_sorted, perm_indices,
 *                                recv_tokens_per_exp
 *   mxmoe_moe_quant_act ........ quant_act_kernel launched by quant_inp_act (:434-592)
 *   mxmoe_moe_silu_mul_quant ... silu_mul_then_quant_kernel launched by silu_mul_then_quant (:595-757)
 *   mxmoe_moe_combine .......... gg_unpermute_out (:66, an empty stub in the reference)
 * The reference's device kernels (act_kernel.cuh) are not in its tree; the arithmetic here is the
 * reference's quant_weight (quantize.cuh:218-279) applied per token row (or 128-element group) and
 * pack_wxax (quantize.cuh:425-475), producing exactly the A operands the GroupGEMM consumes.
 *
 * Conventions: all pointers are DEVICE pointers unless stated; every call is one or two kernel
 * launches on `stream` (hipStream_t as void*), no allocation, no synchronisation; int status
 * (MXMOE_GG_OK == 0; messages via mxmoe_gg_last_error()).
 */
#ifndef MXMOE_MOE_H_
#define MXMOE_MOE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Quantisation tag of one expert's activation (the reference's cvt_qparams_to_tag, ref_bind.cu:467-479). */
enum {
  MXMOE_ACT_FP16 = 0,    /* a_bits 16: the row is copied                                  */
  MXMOE_ACT_INT8 = 1,    /* a_bits 8, one scale per token                                 */
  MXMOE_ACT_INT4 = 2,    /* a_bits 4, one scale per token                                 */
  MXMOE_ACT_INT4_G128 = 3 /* a_bits 4, one scale per (token, 128-element group)           */
};

/* One expert's segment of a permuted activation buffer. Slots (rows of the permuted batch) are
 * sorted by expert; segment e holds slots [first_slot, first_slot + rows). The shared expert, if
 * any, is segment E, fed by every token once (slots T*topk + t). */
typedef struct mxmoe_moe_seg {
  int32_t qtag;        /* MXMOE_ACT_*                                                          */
  int32_t first_slot;  /* first slot of the segment                                           */
  int32_t rows;        /* tokens routed to this expert                                        */
  int32_t width;       /* elements per row of this segment's output (K of the next GEMM)      */
  int64_t out_off;     /* byte offset of the segment's [rows][width * bits / 8] block in `out` */
  int64_t scale_off;   /* fp16-element offset of its scales: [rows] or [width/128][rows]      */
} mxmoe_moe_seg;

/* Stable counting sort of the T*topk expert ids (int32, row-major [T][topk], values in [0, E)):
 *   sorted_expert[s] = expert of slot s (non-decreasing), perm_token[s] = source token of slot s,
 *   inv_slot[t*topk + k] = slot of (token t, choice k), counts[e] = tokens routed to expert e.
 * Equal to torch.sort(topk_ids.view(-1), stable=True) + floor_divide(topk) + bincount(E).
 * One workgroup per expert; E <= 4096. */
int mxmoe_moe_route(const int32_t* topk_ids, int64_t T, int topk, int E, int32_t* sorted_expert,
                    int32_t* perm_token, int32_t* inv_slot, int32_t* counts, void* stream);

/* Gather + quantise the permuted activations: slot s < T*topk reads hidden[perm_token[s]] and is
 * written to segment sorted_expert[s]; with_shared != 0 adds slots T*topk + t, which read hidden[t]
 * into the last segment (nseg - 1: the shared expert). hidden: fp16 [T][K]; segs: DEVICE array of nseg segments, every
 * width == K. Quantised rows: RTN sym in fp16 (scale = fp16(amax / qmax), 0 -> 1;
 * q = rint_even(clamp(fp16(x / scale), +-qmax))), packed per pack_wxax.
 * K % 128 == 0 and K <= 16384. */
int mxmoe_moe_quant_act(const void* hidden, int64_t T, int K, int topk, int with_shared,
                        const int32_t* sorted_expert, const int32_t* perm_token, const mxmoe_moe_seg* segs, int nseg,
                        void* out, void* scales, void* stream);

/* act = fp16_rn(silu(f32 g) * f32 u) of the gate_up output (silu(g) = g * rcp(1 + exp2(-g log2 e)) with
 * the hardware exp2 / reciprocal), then quantised as mxmoe_moe_quant_act.
 * routed_in: fp16 [T*topk][2*N] (slot order; gate = columns [0, N), up = [N, 2N));
 * shared_in: fp16 [T][2*N_shared] or NULL (non-NULL: slots T*topk + t, segment nseg - 1). Segment widths: N for routed experts,
 * N_shared for the shared one (both multiples of 128, <= 16384). */
int mxmoe_moe_silu_mul_quant(const void* routed_in, const void* shared_in, int64_t T, int topk, int N, int N_shared,
                             const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg, void* out,
                             void* scales, void* stream);

/* mxmoe_moe_silu_mul_quant on a gate_up output computed with gate / up rows interleaved in 16-row
 * blocks (MXMOE_GG_EPI_SILU_MUL's weight layout) but the plain epilogue: routed_in [T*topk][2 N],
 * shared_in [T][2 N_shared], columns [32 b, 32 b + 16) = gate columns [16 b, 16 b + 16) and
 * [32 b + 16, 32 b + 32) the matching up columns. Same arithmetic and outputs as
 * mxmoe_moe_silu_mul_quant on the de-interleaved input (the small-batch form of a fused layer). */
int mxmoe_moe_silu_mul_quant_il(const void* routed_in, const void* shared_in, int64_t T, int topk, int N,
                                int N_shared, const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg,
                                void* out, void* scales, void* stream);

/* mxmoe_moe_silu_mul_quant's quantisation alone, for activations the gate_up GroupGEMM already
 * produced with its fused SiLU epilogue (MXMOE_GG_EPI_SILU_MUL, include/mxmoe_gg.h): routed_in fp16
 * [T*topk][N] in slot order, shared_in fp16 [T][N_shared] or NULL; same segments, outputs and limits.
 * (No reference counterpart: the reference's silu_mul_then_quant, ref_bind.cu:595-757, does both.) */
int mxmoe_moe_quant_slots(const void* routed_in, const void* shared_in, int64_t T, int topk, int N, int N_shared,
                          const int32_t* sorted_expert, const mxmoe_moe_seg* segs, int nseg, void* out, void* scales,
                          void* stream);

/* out[t][h] = fp16_rn(acc), acc = +0 then, for k = 0..topk-1 in order,
 *   acc = fma(weights[t][k], f32(y[inv_slot[t*topk + k]][h]), acc),
 * then, if shared != NULL, acc = fma(shared_w ? shared_w[t] : 1, f32(shared[t][h]), acc).
 * y: fp16 [T*topk][H] in slot order; weights: f32 [T][topk]; shared: fp16 [T][H]; H % 8 == 0. */
int mxmoe_moe_combine(const void* y, const int32_t* inv_slot, const float* weights, const void* shared,
                      const float* shared_w, int64_t T, int topk, int H, void* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MXMOE_MOE_H_ */
