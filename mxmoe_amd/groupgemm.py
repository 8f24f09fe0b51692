"""Host-side mirror of the reference GroupGEMM operator interface, on the HIP C-ABI.

Reference interface mirrored (SeaCatComplexes/MxMoE):
  * per-problem QParams {qbits=(a_bits, w_bits), gsize, sym} ..... quantize.cuh:14-25
    (+ the operand format of the reference's fp8 / bf16 strategies: QConfig USE_FP, MMA_E4M3_K32,
    MMA_BF16_FP32 — tile_config.py:40-106, 192)
  * the host API groupgemm_hz_fused_<i>(ptr_As, ptr_Bs, ptr_scale_a, ptr_scale_b, ptr_Cs, ...,
    problem_sizes, qbits_list, problem_count) ...................... kernel_sketch.py:25-46, 82-145
  * the kernel registry (name -> FuncType), registry.cuh:72-107 .... ``registry()``
  * "quant type not supported" for an uncompiled qcfg .............. compose_kernel.py:433

Differences by design: the tile table is planned once into a caller-owned device workspace
(``GroupGemm``), launches are allocation/sync free and run on the caller's stream (torch's
current stream by default), and errors raise ``GGError`` instead of exiting the process.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import torch

from . import _native as nat


FMT_CODES = {"": nat.FMT_DEFAULT, "E4M3": nat.FMT_E4M3, "bf16": nat.FMT_BF16, "F6": nat.FMT_F6}


@dataclasses.dataclass(frozen=True)
class QParams:
    """Per-problem quantisation parameters (reference QParams, quantize.cuh:14-25).

    ``fmt``: "" (fp16 / two's-complement integers), "E4M3" (w8a8_g-1_sym_E4M3: OCP fp8 codes),
    "bf16" (16-bit bfloat16 operands) or "F6" (w4a4_g-1_sym with A and B as fp6 images of the int4
    codes, ``_native.pack_f6``: same results on the fp6 MFMA — lab library only, measured slower
    than the int4 path). The reference's ``_accfp16`` strategies (fp16 MMA with an fp16
    accumulator, tile_config.py:94-97) run as their f32-accumulating base type: MFMA has no fp16
    accumulator, and the f32 sum is the more accurate result of the same products."""

    a_bits: int = 16
    w_bits: int = 16
    gsize: int = -1
    sym: bool = True
    fmt: str = ""

    def __post_init__(self):
        if self.fmt not in FMT_CODES:
            raise ValueError(f"unknown operand format {self.fmt!r}")

    @property
    def is_quant(self) -> bool:
        return self.a_bits < 16 or self.w_bits < 16

    @property
    def is_fp8(self) -> bool:
        return self.fmt == "E4M3"

    @property
    def fmt_code(self) -> int:
        return FMT_CODES[self.fmt]

    @property
    def is_weight_only(self) -> bool:
        """WxA16: fp16 A, quantised B (scale / zp per column or group), cta_gemm.cuh:112-421."""
        return self.a_bits == 16 and self.w_bits < 16

    @property
    def qcfg(self) -> str:
        if not self.is_quant:
            return "bf16" if self.fmt == "bf16" else "fp16"
        return f"w{self.w_bits}a{self.a_bits}_g{self.gsize}_{'sym' if self.sym else 'asym'}" + \
            ("_E4M3" if self.is_fp8 else "_F6" if self.fmt == "F6" else "")

    @staticmethod
    def from_qcfg(qcfg: str) -> "QParams":
        """Any SUPPORTED_QCFG string (tile_config.py:40-59); ``_accfp16`` maps to its base type."""
        if qcfg in ("fp16", "fp16_accfp16"):
            return QParams()
        if qcfg == "bf16":
            return QParams(fmt="bf16")
        w = int(qcfg.split("w")[1].split("a")[0])
        a = int(qcfg.split("a")[1].split("_g")[0])
        g = int(qcfg.split("_g")[1].split("_")[0])
        if qcfg.endswith("_bf16"):
            raise ValueError(f"{qcfg}: weight-only with bf16 activations is not built on MI355X")
        fmt = "E4M3" if qcfg.endswith("_E4M3") else "F6" if qcfg.endswith("_F6") else ""
        return QParams(a_bits=a, w_bits=w, gsize=g, sym="asym" not in qcfg, fmt=fmt)


FP16 = QParams()
BF16 = QParams(fmt="bf16")
W8A8 = QParams(8, 8, -1, True)
W8A8_E4M3 = QParams(8, 8, -1, True, "E4M3")  # w8a8_g-1_sym_E4M3: OCP fp8 operands, f32 accumulate
W4A4 = QParams(4, 4, -1, True)
W4A4_F6 = QParams(4, 4, -1, True, "F6")  # w4a4_g-1_sym on fp6 images (lab library: nat.pack_f6 of A and B)
W4A4_G128 = QParams(4, 4, 128, True)  # w4a4_g128_sym: one scale per 128-K group (cta_gemm.cuh:610-772)
# weight-only (any group size that is -1 or a multiple of 64 dividing K, sym or asym, 2 / 4 / 8 bits)
W4A16_G128_ASYM = QParams(16, 4, 128, False)
W4A16_ASYM = QParams(16, 4, -1, False)
W4A16_G128_SYM = QParams(16, 4, 128, True)
W8A16_ASYM = QParams(16, 8, -1, False)
W2A16_G128_ASYM = QParams(16, 2, 128, False)

SUPPORTED = {q.qcfg: q for q in (FP16, BF16, W8A8, W8A8_E4M3, W4A4, W4A4_G128, W4A16_G128_ASYM, W4A16_ASYM, W4A16_G128_SYM, W8A16_ASYM,
                                  QParams(16, 4, -1, True), QParams(16, 8, -1, True), QParams(16, 8, 128, True),
                                  QParams(16, 8, 128, False), W2A16_G128_ASYM, QParams(16, 2, -1, False),
                                  QParams(16, 2, -1, True), QParams(16, 2, 128, True))}


@dataclasses.dataclass
class Problem:
    """One GroupGEMM problem  C[M,N] = A[M,K] . B[N,K]^T  on device tensors.

    fp16 / bf16: A [M,K], B [N,K] 16-bit.  quant (incl. E4M3 codes): A uint8 [M, K*a_bits/8] / B uint8 [N, K*w_bits/8]
    in pack_wxax layout, scale_a fp16 [M], scale_b fp16 [N] (w4a4_g128: [K/128][M] and [K/128][N],
    the permute_scale layout).  C fp16 [M, ldc] (ldc >= N).
    """

    A: torch.Tensor
    B: torch.Tensor
    C: torch.Tensor
    M: int
    N: int
    K: int
    q: QParams = FP16
    scale_a: Optional[torch.Tensor] = None
    scale_b: Optional[torch.Tensor] = None
    lda: int = 0  # row strides in 16-bit words, 0 = dense
    ldb: int = 0
    ldc: int = 0
    # fused SiLU epilogue (MXMOE_GG_EPI_SILU_MUL): B rows gate / up interleaved in 16-row blocks
    # (interleave_gate_up), C [M, N/2] = silu(gate) * up — fp16 / w8a8 / w4a4, large-batch kernels
    silu: bool = False

    def __post_init__(self):
        """Operand dtypes must match q's format: the C-ABI sees only bytes, so an fp16 operand
        labelled bf16 (or float data labelled as integer codes) would run and return garbage."""
        def need(t, ok, what):
            if t is not None and t.numel() > 0 and t.dtype not in ok:  # (empty: a planning placeholder)
                raise ValueError(f"{self.q.qcfg}: {what} must be {' / '.join(map(str, ok))}, got {t.dtype}")

        codes = (torch.uint8, torch.int8, torch.int16, torch.uint16, torch.int32, torch.float8_e4m3fn)
        if self.q.fmt == "bf16":
            need(self.A, (torch.bfloat16,), "A")
            need(self.B, (torch.bfloat16,), "B")
        elif not self.q.is_quant:
            need(self.A, (torch.float16,), "A")
            need(self.B, (torch.float16,), "B")
        else:
            need(self.A, (torch.float16,) if self.q.is_weight_only else codes, "A")
            need(self.B, codes, "B (packed codes)")
        need(self.C, (torch.float16,), "C")

    def to_c(self) -> nat.GGProblemC:
        def ptr(t):
            return 0 if t is None else t.data_ptr()

        return nat.GGProblemC(
            A=ptr(self.A), B=ptr(self.B), scale_a=ptr(self.scale_a), scale_b=ptr(self.scale_b), C=ptr(self.C),
            M=self.M, N=self.N, K=self.K, a_bits=self.q.a_bits, w_bits=self.q.w_bits, gsize=self.q.gsize,
            sym=int(self.q.sym), fmt=self.q.fmt_code | (nat.EPI_SILU_MUL if self.silu else 0), lda=self.lda,
            ldb=self.ldb, ldc=self.ldc)

    @property
    def flops(self) -> int:
        return 2 * self.M * self.N * self.K


def interleave_gate_up(w: torch.Tensor, scale: Optional[torch.Tensor] = None, rows_per_row: int = 1):
    """Gate / up rows of a [2N, ...] gate_up weight (gate rows first, then up rows) reordered for the
    fused SiLU epilogue: 16-row blocks alternating gate block b, up block b. ``rows_per_row``: rows of
    ``w`` per weight row (1 for the [N][K] layouts here). Returns (w', scale') — scale (per row,
    [2N]) permuted alike. Done once per weight, like the weight-only repack."""
    n2 = w.shape[0] // rows_per_row
    if n2 % 32:
        raise ValueError("interleave_gate_up: 2N must be a multiple of 32")
    n = n2 // 2
    idx = torch.arange(n2, device=w.device).view(2, n // 16, 16).transpose(0, 1).reshape(-1)
    w2 = w.view(n2, rows_per_row, *w.shape[1:]).index_select(0, idx).reshape(w.shape)
    return w2, (None if scale is None else scale.index_select(0, idx))


def registry() -> list[str]:
    """Compiled kernel variants (the reference's GetGlobalRegistry(), registry.cuh:99-102)."""
    return nat.list_variants()


def _stream_handle(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class GroupGemm:
    """A planned GroupGEMM: the tile table lives in a device workspace owned by this object.

    ``launch()`` is a single kernel launch on the given (or current) stream; it performs no
    allocation and no host synchronisation, so it can be captured in a CUDA/HIP graph.
    """

    def __init__(self, problems: Sequence[Problem], variant: Optional[int] = None,
                 device: Optional[torch.device] = None, stream: Optional[torch.cuda.Stream] = None):
        self.problems = list(problems)
        # None -> MXMOE_GG_VARIANT_AUTO (-1): the library picks by quant-type mix; after planning
        # self.variant is the concrete variant
        self.variant = nat.VARIANT_AUTO if variant is None else int(variant)
        if device is None:
            device = self.problems[0].C.device if self.problems else torch.device("cuda")
        self.device = device
        for p in self.problems:
            for t in (p.A, p.B, p.C, p.scale_a, p.scale_b):
                if t is not None and t.device != device:
                    raise ValueError(f"all tensors must live on {device}, got {t.device}")
        P = len(self.problems)
        self._c_problems = (nat.GGProblemC * max(P, 1))(*[p.to_c() for p in self.problems])
        ws_bytes = nat.workspace_size(self._c_problems, P, self.variant)
        self.workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
        self.info = nat.GGPlanInfo()
        nat.check(nat.lib().mxmoe_gg_plan(self._c_problems, P, self.variant, ctypes.c_void_p(self.workspace.data_ptr()),
                                          ws_bytes, ctypes.c_void_p(_stream_handle(stream)), ctypes.byref(self.info)))
        self.variant = int(self.info.variant)

    @property
    def total_tiles(self) -> int:
        return self.info.total_tiles

    @property
    def flops(self) -> int:
        return sum(p.flops for p in self.problems)

    def rebind(self, problems: Sequence[Problem], stream: Optional[torch.cuda.Stream] = None) -> None:
        """Point the plan at new operand buffers of the same shapes / quant params / strides
        (mxmoe_gg_rebind: uploads the pointer columns only; GGError if the shapes differ)."""
        problems = list(problems)
        for p in problems:
            for t in (p.A, p.B, p.C, p.scale_a, p.scale_b):
                if t is not None and t.device != self.device:
                    raise ValueError(f"all tensors must live on {self.device}, got {t.device}")
        P = len(problems)
        cps = (nat.GGProblemC * max(P, 1))(*[p.to_c() for p in problems])
        nat.check(nat.lib().mxmoe_gg_rebind(cps, P, ctypes.byref(self.info), ctypes.c_void_p(_stream_handle(stream))))
        self.problems, self._c_problems = problems, cps

    def __del__(self):
        # the workspace is freed with this object: drop the library's rebind key for its address
        ws = getattr(self, "workspace", None)
        if ws is not None and nat._lib is not None:
            try:
                nat._lib.mxmoe_gg_forget_workspace(ctypes.c_void_p(ws.data_ptr()))
            except Exception:  # pragma: no cover - interpreter shutdown
                pass

    def launch(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        nat.check(nat.lib().mxmoe_gg_launch(ctypes.byref(self.info), ctypes.c_void_p(_stream_handle(stream))))

    __call__ = launch


def group_gemm(problems: Sequence[Problem], variant: Optional[int] = None,
               stream: Optional[torch.cuda.Stream] = None) -> None:
    """Plan + launch once (the reference host API's per-call behaviour)."""
    GroupGemm(problems, variant=variant, stream=stream).launch(stream)


def groupgemm_reference_abi(ptr_As: torch.Tensor, ptr_Bs: torch.Tensor, ptr_scale_a: torch.Tensor,
                            ptr_scale_b: torch.Tensor, ptr_Cs: torch.Tensor, h_problem_sizes: Sequence[tuple],
                            h_qbits_list: Sequence[QParams], pad_byte: int = 0) -> None:
    """Call the drop-in ``groupgemm_mxmoe`` entry (reference FuncType, registry.cuh:28-39).

    ``ptr_*`` are int64 device tensors holding device pointers (the reference's device arrays).
    ``pad_byte`` fills the three padding bytes of every QParams (the reference leaves them
    uninitialised; the library must ignore them). Problems with a non-default operand format (E4M3,
    bf16 — not expressible in the reference's QParams) go through ``groupgemm_mxmoe_fmt``.
    """
    P = len(h_problem_sizes)
    dims = (nat.MxmoeDim3 * max(P, 1))(*[nat.MxmoeDim3(int(m), int(n), int(k)) for (m, n, k) in h_problem_sizes])
    qps = (nat.MxmoeQParams * max(P, 1))(
        *[nat.MxmoeQParams(q.a_bits, q.w_bits, q.gsize, int(q.sym), (ctypes.c_uint8 * 3)(pad_byte, pad_byte, pad_byte))
          for q in h_qbits_list])
    dev_dims = torch.tensor([[m, n, k] for (m, n, k) in h_problem_sizes], dtype=torch.int32, device=ptr_As.device)
    args = (ptr_As.data_ptr(), ptr_Bs.data_ptr(), ptr_scale_a.data_ptr(), ptr_scale_b.data_ptr(), ptr_Cs.data_ptr(),
            None, None, None, None, None, ctypes.c_void_p(dev_dims.data_ptr()), dims, None, qps, P)
    if any(q.fmt_code != nat.FMT_DEFAULT for q in h_qbits_list):
        fmts = (ctypes.c_int32 * max(P, 1))(*[q.fmt_code for q in h_qbits_list])
        nat.check(nat.lib().groupgemm_mxmoe_fmt(*args, fmts))
    else:
        nat.check(nat.lib().groupgemm_mxmoe(*args))
