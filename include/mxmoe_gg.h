/*
 * mxmoe_gg.h — C-ABI of the MI355X (gfx950) mixed-precision MoE GroupGEMM.
 *
 * One call computes P independent problems  C_i[M_i,N_i] = A_i[M_i,K_i] . B_i[N_i,K_i]^T
 * (RCR layout: A row-major, B "column-major" = [N][K] with K contiguous, C row-major fp16),
 * each problem with its own quantisation type:
 *
 *   fp16 : A,B fp16, fp32 accumulate, C = fp16_rn(acc)
 *   w8a8 : A,B int8  per-channel sym (gsize -1), exact int32 accumulate,
 *          C = fp16_rn(0.f + f32(acc) * f32(fp16_rn(sa[m] * sb[n])))
 *   w4a4 : A,B int4  per-channel sym (gsize -1), same epilogue
 *   w4a4_g128, WxA16 weight-only: see DESIGN.md §4 / mxmoe_gg_repack_weightonly below
 *   w8a8_g-1_sym_E4M3 (fmt MXMOE_GG_FMT_E4M3): A,B OCP fp8 e4m3 codes (one byte each, pack_wxax
 *          8-bit byte order), per-channel fp16 scales, f32 accumulate (products exact, sum order
 *          unspecified), C = fp16_rn(0.f + acc * f32(fp16_rn(sa[m] * sb[n])))
 *   bf16 (fmt MXMOE_GG_FMT_BF16): A,B bf16, fp32 accumulate, C = fp16_rn(acc) (C is fp16 for every
 *          type, as the reference's `half** ptr_Cs`)
 *
 * Data layout is byte-identical to the reference bench (SeaCatComplexes/MxMoE):
 *   - packed A/B words follow pack_wxax        (mxmoe/kernels/src/include/quantize.cuh:425-475)
 *   - QParams {int2 qbits(x=a_bits,y=w_bits); int gsize; bool sym}  (quantize.cuh:14-25)
 *   - scale_a[M], scale_b[N] fp16 per problem  (test.cu:301-313, 522-523)
 *   - epilogue arithmetic                      (mm_tile.cuh:469-496, 610-662; cta_gemm.cuh:599-607)
 *
 * Conventions (differences from the reference ABI):
 *   - every entry point returns an int status (MXMOE_GG_OK == 0); nothing calls exit();
 *     mxmoe_gg_last_error() returns a thread-local message for the last failure;
 *   - the caller owns all device memory, including the workspace; no call allocates
 *     device memory except the reference-compatible shim groupgemm_mxmoe();
 *   - explicit stream argument (hipStream_t passed as void*); mxmoe_gg_launch() does no host
 *     synchronisation and no allocation, so it can be captured into a hipGraph;
 *   - mutable global state: the thread-local error string, the reference shim's per-device
 *     workspaces (mxmoe_gg_release_shim_workspaces) and mxmoe_gg_rebind's per-workspace plan keys
 *     (mutex-guarded, host memory only).
 */
#ifndef MXMOE_GG_H_
#define MXMOE_GG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MXMOE_GG_ABI_VERSION 7  /* 5: QParams padding ignored, groupgemm_mxmoe_fmt; 6: MXMOE_GG_EPI_SILU_MUL;
                                 * 7: mxmoe_gg_variant_caps */

enum {
  MXMOE_GG_OK = 0,
  MXMOE_GG_ERR_INVALID = 1,     /* bad argument / shape / alignment */
  MXMOE_GG_ERR_UNSUPPORTED = 2, /* quantisation type or variant not compiled */
  MXMOE_GG_ERR_WORKSPACE = 3,   /* workspace too small */
  MXMOE_GG_ERR_HIP = 4          /* a HIP runtime call failed */
};

/* Element format of a problem's A / B beyond the bit widths (the reference's QConfig USE_FP flag,
 * tile_config.py:192, and its MMA_BF16_FP32 / MMA_E4M3_K32 strategies, tile_config.py:87-106). */
enum {
  MXMOE_GG_FMT_DEFAULT = 0, /* fp16 for 16-bit operands, two's-complement integers otherwise */
  MXMOE_GG_FMT_E4M3 = 1,    /* w8a8_g-1_sym_E4M3: OCP fp8 e4m3 codes                         */
  MXMOE_GG_FMT_BF16 = 2     /* bf16: 16-bit operands are bfloat16                              */
};

/* Epilogue flag, OR-ed into mxmoe_gg_problem.fmt (fp16, w8a8_g-1_sym and w4a4_g-1_sym problems on the
 * v2x, v3 and wo3 variants; weight-only WxA16 problems on wo3, whose scale_b is permuted with the rows;
 * no reference counterpart — it fuses the MoE layer's silu_mul_then_quant
 * activation, ref_bind.cu:595-757, into the gate_up GroupGEMM). B holds N = 2 Nh rows interleaved
 * in 16-row blocks: rows [32 b, 32 b + 16) are gate rows [16 b, 16 b + 16) and rows
 * [32 b + 16, 32 b + 32) the matching up rows (scale_b permuted alike; N % 32 == 0). C is [M][Nh]
 * (ldc >= Nh, 0 = Nh): C[m][n] = fp16_rn(silu(f32 g) * f32 u) with g, u the fp16 outputs the call
 * would have written for gate column n and up column n, silu(g) = g * rcp(1 + exp2(-g log2 e)) —
 * the arithmetic of mxmoe_moe_silu_mul_quant, bit for bit. */
#define MXMOE_GG_EPI_SILU_MUL 0x100

/* Same memory layout as the reference's mxmoe::QParams (quantize.cuh:14-25):
 * int2 qbits {x = a_bits, y = w_bits}; int gsize; bool sym; padded to 16 bytes, 8-byte aligned.
 * The three bytes after `sym` are the reference's padding: its QParams constructors
 * (quantize.cuh:19-20) leave them uninitialised, so nothing in this library reads them. Operand
 * formats other than the default travel in mxmoe_gg_problem.fmt or groupgemm_mxmoe_fmt's array. */
typedef struct mxmoe_qparams {
  int32_t a_bits;
  int32_t w_bits;
  int32_t gsize;
  uint8_t sym;
  uint8_t pad_[3];
} __attribute__((aligned(8))) mxmoe_qparams;

/* Same memory layout as CUDA/HIP dim3 (x = M, y = N, z = K), as used in registry.cuh:28-39. */
typedef struct mxmoe_dim3 {
  uint32_t x, y, z;
} mxmoe_dim3;

/* One GroupGEMM problem (host-side descriptor). Pointers are DEVICE pointers.
 * lda/ldb/ldc are row strides in 16-bit words (the reference's `half` unit); 0 = dense. */
typedef struct mxmoe_gg_problem {
  const void* A;       /* fp16 [M][K]  or packed [M][K*a_bits/16] words            */
  const void* B;       /* fp16 [N][K]  or packed [N][K*w_bits/16] words            */
  const void* scale_a; /* fp16 [M] (quantised problems only, else may be NULL)     */
  const void* scale_b; /* fp16 [N] (quantised problems only, else may be NULL)     */
  void* C;             /* fp16 [M][ldc]                                            */
  int32_t M, N, K;
  int32_t a_bits, w_bits, gsize, sym;
  int32_t fmt; /* MXMOE_GG_FMT_* */
  int64_t lda, ldb, ldc;
} mxmoe_gg_problem;

/* Result of planning: what mxmoe_gg_launch needs on the host side. */
typedef struct mxmoe_gg_plan_info {
  int32_t variant;
  int32_t problem_count;
  int32_t total_tiles;
  int32_t grid;
  int32_t block;
  int32_t lds_bytes;
  int32_t qtype_mask;      /* bit q set if a planned problem has quant type q (0 fp16, 1 w8a8, 2 w4a4,
                            * 3 w4a16, 4 w8a16, 5 w4a4_g128, 6 w2a16, 7 w8a8 E4M3, 8 bf16); bit 16:
                            * a weight-only problem carries MXMOE_GG_EPI_SILU_MUL (small-batch kernel);
                            * selects the kernel specialisation at launch */
  int32_t splitk_slabs;    /* 256-KiB partial-sum slabs the plan's split-K tiles use (0: no split) */
  int64_t workspace_bytes; /* bytes of the workspace actually used by the plan */
  void* workspace;         /* device workspace the plan was written to */
  uint64_t signature;      /* hash of the plan table and tile table (shapes, quant params, strides) */
  int32_t tile_slots;      /* entries of the device tile table (= grid, except for persistent variants,
                            * whose workgroups walk [k][grid]-ordered tile lists) */
  int32_t reserved;
} mxmoe_gg_plan_info;

int mxmoe_gg_abi_version(void);

/* Thread-local message describing the last failed call on this thread ("" if none). */
const char* mxmoe_gg_last_error(void);

/* Number of compiled kernel variants. */
int mxmoe_gg_variant_count(void);

/* The variant AUTO resolves to for long-K calls that are not w4a4-only (mxmoe_gg_resolve_variant). */
int mxmoe_gg_default_variant(void);

/* Writes a newline-separated description of every compiled variant into buf (truncated,
 * always NUL-terminated when n > 0). Line i describes variant i in the reference TileConfig
 * repr form per qcfg, e.g. "0 fused fp16=TileConfig(BM=128, BN=128, ...) w8a8_g-1_sym=...".
 * Returns the number of variants, or a negative status on error. */
int mxmoe_gg_list_variants(char* buf, size_t n);

/* Tile geometry of variant `variant` for a quantisation type (a_bits, w_bits):
 * writes BM, BN, K-bytes-per-stage and threads per workgroup. */
int mxmoe_gg_variant_tile(int variant, int a_bits, int w_bits, int32_t* bm, int32_t* bn, int32_t* bk_bytes,
                          int32_t* threads);

/* Capability bits of a compiled variant (mxmoe_gg_variant_caps). */
#define MXMOE_GG_CAP_SILU_MUL 1u /* plans problems carrying MXMOE_GG_EPI_SILU_MUL (the fused SiLU epilogue) */

/* Capabilities of variant `variant` (an index, not AUTO): *caps = OR of MXMOE_GG_CAP_* bits. Lets a
 * caller ask whether the kernel AUTO resolved to supports an epilogue before planning with it
 * (the MoE layer routes small-batch gate_up calls, whose kernel has no SiLU epilogue, through the
 * interleaved SiLU pass). No reference counterpart: the reference compiles one epilogue per kernel. */
int mxmoe_gg_variant_caps(int variant, uint32_t* caps);

/* Pass as `variant` to mxmoe_gg_workspace_size / _plan / _run: the library picks the variant
 * from the quant types present (the plan info records the concrete one). groupgemm_mxmoe uses it. */
#define MXMOE_GG_VARIANT_AUTO (-1)

/* The concrete variant `variant` (MXMOE_GG_VARIANT_AUTO or an index) resolves to for these
 * problems, written to *out. Host only (no GPU). AUTO: small-batch calls (mean rows per weight
 * byte under the DESIGN.md §4 cuts) -> the 3-WG/CU 64-row kernel (wo3); w4a4-only sets -> the
 * 256x128 2-WG/CU kernel (unless the plan needs split-K); otherwise mxmoe_gg_default_variant(). */
int mxmoe_gg_resolve_variant(const mxmoe_gg_problem* problems, int problem_count, int variant, int* out);

/* Device workspace bytes the plan of these problems needs with this variant
 * (plan table + pointer arrays + tile table). Validates the problems like mxmoe_gg_plan. */
int mxmoe_gg_workspace_size(const mxmoe_gg_problem* problems, int problem_count, int variant, size_t* bytes);

/* Validate problems, build the tile table and upload it into the workspace (hipMemcpyAsync on
 * `stream`, then a stream synchronisation: planning is done once, outside the hot loop).
 * The host problem array may be freed after return. */
int mxmoe_gg_plan(const mxmoe_gg_problem* problems, int problem_count, int variant, void* workspace,
                  size_t workspace_bytes, void* stream, mxmoe_gg_plan_info* info);

/* Re-point a plan at new operand buffers: `problems` must describe the same shapes, quant params
 * and strides as the planned call (checked through the plan signature, MXMOE_GG_ERR_INVALID
 * otherwise); only the 5 pointer columns of the workspace are uploaded (one copy on `stream` and a
 * stream synchronisation). The pointers get mxmoe_gg_plan's NULL / alignment checks.
 * BLOCKING and NOT graph-capturable (unlike mxmoe_gg_launch): the call ends with
 * hipStreamSynchronize(stream). The library remembers, per workspace, a key over the planned
 * shapes / quant params / strides: a rebind with the same key skips the host planner (pointers are
 * still checked); otherwise the planner re-runs to compare the plan signature. A plan must be
 * rebound on the stream its launches run on: the upload is ordered behind that stream's work only. */
int mxmoe_gg_rebind(const mxmoe_gg_problem* problems, int problem_count, const mxmoe_gg_plan_info* info, void* stream);

/* Drop mxmoe_gg_rebind's remembered plan key for `workspace` (call before freeing a workspace that
 * held a plan; host only, no device access). A later plan into the same address re-registers it.
 * Returns MXMOE_GG_OK whether or not an entry existed. */
int mxmoe_gg_forget_workspace(const void* workspace);

/* Launch a planned GroupGEMM on `stream`. No allocation, no synchronisation. */
int mxmoe_gg_launch(const mxmoe_gg_plan_info* info, void* stream);

/* plan + launch. */
int mxmoe_gg_run(const mxmoe_gg_problem* problems, int problem_count, int variant, void* workspace,
                 size_t workspace_bytes, void* stream);

/* Drop-in for the reference registry FuncType (mxmoe/kernels/src/include/registry.cuh:28-39;
 * generated host API groupgemm_hz_fused_<i>, kernel_sketch.py:25-46, 82-145).
 * ptr_* / problem_sizes / qbits_list are DEVICE arrays, h_problem_sizes / h_qbits_list host
 * copies; ptr_Ds and the ld* arrays are accepted and ignored exactly as in the reference.
 * Runs the AUTO variant on the legacy default stream. Unlike the reference it reports errors
 * through the return value (and mxmoe_gg_last_error) instead of exit(), and validates the gathered
 * device pointers (NULL, 16-B alignment) like mxmoe_gg_plan. It keeps one workspace and one pinned
 * staging buffer per device (grown on demand, one host synchronisation per call); release them with
 * mxmoe_gg_release_shim_workspaces(). */
int groupgemm_mxmoe(void** ptr_As, void** ptr_Bs, void** ptr_scale_a, void** ptr_scale_b, void** ptr_Cs,
                    void** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                    mxmoe_dim3* problem_sizes, mxmoe_dim3* h_problem_sizes, mxmoe_qparams* qbits_list,
                    mxmoe_qparams* h_qbits_list, int problem_count);

/* groupgemm_mxmoe with an explicit operand format per problem (h_fmts[i] = MXMOE_GG_FMT_*, host
 * array; NULL = MXMOE_GG_FMT_DEFAULT for every problem, i.e. exactly groupgemm_mxmoe). The opt-in
 * for the E4M3 / bf16 strategies, which the reference's QParams cannot express. */
int groupgemm_mxmoe_fmt(void** ptr_As, void** ptr_Bs, void** ptr_scale_a, void** ptr_scale_b, void** ptr_Cs,
                        void** ptr_Ds, int64_t* ldas, int64_t* ldbs, int64_t* ldcs, int64_t* ldds,
                        mxmoe_dim3* problem_sizes, mxmoe_dim3* h_problem_sizes, mxmoe_qparams* qbits_list,
                        mxmoe_qparams* h_qbits_list, int problem_count, const int32_t* h_fmts);

/* Free groupgemm_mxmoe's per-device workspaces and staging buffers (waits for each device to be
 * idle first). Safe to call at any time; the next shim call re-allocates. */
int mxmoe_gg_release_shim_workspaces(void);

/* Weight-only (WxA16) B, host-side and once per weight: converts the reference's packed words
 * (pack_weightonly after permute_weight(Row), quantize.cuh:318-421: uint16 [N / (16/w_bits)][K],
 * sym codes stored with the +2^(w_bits-1)-1 offset) into the layout the kernels read:
 * uint8 [N][K * w_bits / 8], per 64-K segment of a row the K values {kc*32 + g*8 + e} at element
 * position g*16 + kc*8 + e (kc < 2, g < 4, e < 8); 4-bit: e at nibble (e >> 1) | (e & 1) << 2 of
 * the unit's 32-bit word (codes 2q, 2q+1 at bits 4q and 16 + 4q), low nibble first; 2-bit: the
 * unit (g) of a segment's 16-B row is one little-endian 32-bit word at byte 4 g holding both K
 * halves, code (kc, e) at bit 16 (e & 1) + 2 (4 kc + e / 2). Code values are
 * unchanged. Needs N % (8 * 16 / w_bits) == 0 and K % 64 == 0; w_bits 2, 4 or 8. The scale / zero
 * buffer is used as the reference lays it out (permute_scale: [K/gsize][N] sym, [K/gsize][N][2]
 * scale/zp pairs asym). */
int mxmoe_gg_repack_weightonly(const uint16_t* ref_words, int N, int K, int w_bits, uint8_t* out);

/* Diagnostics (no reference counterpart): the tile timeline the "abl_v2s_trace" variant records,
 * 4 uint64 per block {start, mainloop end, end after its stores drained (s_memrealtime, 100 MHz
 * ticks), K stages << 48 | height class << 40 | qtype << 36 | XCC_ID << 32 | HW_ID} for the first
 * 32768 blocks of the last traced launch. Copies
 * min(bytes, 1 MiB) into host memory `dst` (synchronous); reset != 0 then zeroes the record. */
int mxmoe_gg_debug_trace(void* dst, size_t bytes, int reset);

/* Diagnostics (no reference counterpart): the host tile table mxmoe_gg_plan would upload, without
 * touching a device — 8 int32 per workgroup slot {table row (-1 = empty slot), m0, n0, class
 * (bits 8-15 split-K slice, 16-23 slices), first K stage, end K stage, split-K slab, split-K group},
 * blockIdx order (XCD x runs slots x, x + 8, ...); `rows` (optional, problem_count int32) receives
 * the caller's problem index of every table row. Writes min(*slots, needed) slots and sets *slots
 * to the number needed. */
int mxmoe_gg_plan_tiles(const mxmoe_gg_problem* problems, int problem_count, int variant, int32_t* tiles,
                        int32_t* rows, int* slots);

#ifdef __cplusplus
}
#endif

#endif /* MXMOE_GG_H_ */
