"""Shared helpers for tests: seeded problem construction + oracle expectations."""
from __future__ import annotations

import numpy as np
import torch

from mxmoe_amd import _native as nat
from mxmoe_amd.groupgemm import BF16, FP16, W4A4, W4A4_G128, W8A8, W8A8_E4M3, Problem, QParams
from mxmoe_amd.quantize import pack_e4m3, pack_wxax, quant_e4m3, quant_rtn_sym
from oracle import oracle, weightonly

QCFGS = {"fp16": FP16, "w8a8_g-1_sym": W8A8, "w4a4_g-1_sym": W4A4, "w4a4_g128_sym": W4A4_G128,
         "w8a8_g-1_sym_E4M3": W8A8_E4M3, "bf16": BF16}


FULL_SIZE_CFGS = ("fp16", "w8a8", "w4a4", "mixed", "ds2_mixed")  # BASELINE configs[1]-[4] at bs=8192


def full_size_variants() -> list:
    """Variants the full-size (bs=8192) parity tests run: EVERY production variant, so the kernel
    AUTO hands a benched config to (the kernel of record) is always among them
    (tests/test_abi.py::test_full_size_parity_covers_auto_choices guards this)."""
    return list(nat.production_variants())


def full_size_layer(cfg: str) -> dict:
    """{"gate_up": [QShape], "down": [QShape]} of one BASELINE full-size config."""
    from mxmoe_amd.workload import (ds2_mixed_qconfig, ds2_workload, load_workload, mixed_qconfig_lp1,
                                    qwen2_layer11_workload)

    if cfg == "ds2_mixed":
        return load_workload(ds2_workload(8192, qconfig=ds2_mixed_qconfig()))["layer-1"]
    kw = {"fp16": {}, "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
          "mixed": dict(qconfig=mixed_qconfig_lp1())}[cfg]
    return load_workload(qwen2_layer11_workload(8192, **kw))["layer-11"]


def exact_compare(q: QParams) -> bool:
    """Integer-accumulating quant types are checked bit for bit; fp16 / bf16 / weight-only / E4M3
    (f32 sums in an unspecified order) within the fp16 tolerance."""
    return q.is_quant and not q.is_weight_only and not q.is_fp8


class HostProblem:
    """Host copies of one problem's inputs (numpy) + the device Problem."""

    def __init__(self, M, N, K, q: QParams, seed: int, device: str, ldc: int = 0, C: torch.Tensor | None = None,
                 c_col0: int = 0, ref_format: bool = False):
        g = torch.Generator().manual_seed(seed)
        self.M, self.N, self.K, self.q = M, N, K, q
        a = (torch.rand(M, K, generator=g, dtype=torch.float32) * 2 - 1).to(torch.float16)
        b = (torch.rand(N, K, generator=g, dtype=torch.float32) * 2 - 1).to(torch.float16)
        if q.is_fp8:
            qa, sa = quant_e4m3(a)
            qb, sb = quant_e4m3(b)
            self.qa, self.qb = qa.numpy(), qb.numpy()
            self.A, self.B = pack_e4m3(qa).numpy(), pack_e4m3(qb).numpy()
            self.sa, self.sb = sa.numpy(), sb.numpy()
        elif q.fmt == "bf16":
            self.A = a.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
            self.B = b.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
            self.sa = self.sb = None
        elif q.is_weight_only:
            # oracle quantisation; B either packed straight into the kernel layout or built in the
            # reference's packed format and converted by the library (the drop-in route)
            qv, sz = weightonly.quant_wo(b.numpy(), q.w_bits, q.gsize, q.sym)
            self.sb = weightonly.permute_scale(sz, N, K, q.gsize, q.sym)
            self.qb = qv
            if ref_format:
                self.B = nat.repack_weightonly(weightonly.ref_pack(qv, q.w_bits, q.sym), N, K, q.w_bits)
            else:
                self.B = weightonly.mi355x_pack(qv, q.w_bits, q.sym)
            self.A = a.numpy()
            self.sa = None
        elif q.is_quant:
            bits = q.a_bits
            qa, sa = quant_rtn_sym(a, bits, q.gsize)
            qb, sb = quant_rtn_sym(b, bits, q.gsize)
            self.qa, self.qb = qa.numpy(), qb.numpy()
            self.A = pack_wxax(qa, bits).numpy()
            self.B = pack_wxax(qb, bits).numpy()
            self.sa, self.sb = sa.numpy(), sb.numpy()
        else:
            self.A, self.B = a.numpy(), b.numpy()
            self.sa = self.sb = None
        self.ldc = ldc or N
        dev = torch.device(device)
        if C is None:
            self.Cbuf = torch.full((max(M, 1), self.ldc), float("nan"), dtype=torch.float16, device=dev)
            Cview = self.Cbuf
        else:
            self.Cbuf = C
            Cview = C[:, c_col0:]
        self.c_col0 = c_col0
        if q.fmt == "bf16":
            tA = torch.from_numpy(self.A.view(np.int16)).view(torch.bfloat16).to(dev)
            tB = torch.from_numpy(self.B.view(np.int16)).view(torch.bfloat16).to(dev)
        else:
            tA, tB = torch.from_numpy(self.A).to(dev), torch.from_numpy(self.B).to(dev)
        self.problem = Problem(
            A=tA, B=tB, C=Cview, M=M, N=N, K=K, q=q,
            scale_a=None if self.sa is None else torch.from_numpy(self.sa).to(dev),
            scale_b=None if self.sb is None else torch.from_numpy(self.sb).to(dev),
            ldc=self.ldc if C is None else C.shape[1])

    def expected(self) -> np.ndarray:
        if self.q.is_fp8:
            return oracle.gg_e4m3(self.A, self.B, self.sa, self.sb, self.M, self.N, self.K)
        if self.q.fmt == "bf16":
            return oracle.gg_bf16(self.A, self.B, self.M, self.N, self.K)
        if self.q.is_weight_only:
            q = self.q
            return weightonly.gemm(self.A, weightonly.dequant(self.qb, self.sb, self.N, self.K, q.w_bits, q.gsize, q.sym))
        if self.q.is_quant and self.q.gsize != -1:
            return oracle.gg_quant_grouped(self.A, self.B, self.sa, self.sb, self.M, self.N, self.K, self.q.a_bits,
                                           self.q.gsize)
        if self.q.is_quant:
            return oracle.gg_quant(self.A, self.B, self.sa, self.sb, self.M, self.N, self.K, self.q.a_bits)
        return oracle.gg_f16(self.A, self.B, self.M, self.N, self.K)

    def result(self) -> np.ndarray:
        c = self.problem.C
        return c[: self.M, : self.N].cpu().numpy()


def assert_f16_close(out: np.ndarray, ref: np.ndarray, K: int):
    """fp16 GroupGEMM tolerance: relative 1e-3 (north_star) plus an absolute floor for cancellation,
    |out-ref| <= 1e-3*|ref| + 1e-3*rms(ref) + 2^-10 * (K * 2^-24 * |a||b| bound ~ 0)."""
    out = out.astype(np.float64)
    ref = ref.astype(np.float64)
    assert np.isfinite(out).all(), "non-finite output"
    rms = float(np.sqrt(np.mean(ref * ref))) if ref.size else 0.0
    tol = 1e-3 * np.abs(ref) + 1e-3 * rms + 1e-6
    bad = np.abs(out - ref) > tol
    assert not bad.any(), f"{bad.sum()} / {bad.size} fp16 outputs outside tolerance; max err " \
                          f"{np.max(np.abs(out - ref))}"


def assert_fakequant_close(out: np.ndarray, ref_fq: np.ndarray, what: str = ""):
    """Parity against the reference's executed definition of a quantised linear,
    C_fq = F.linear(Quantizer.fake_quant(a), Quantizer.fake_quant(b)) in fp32 (quant.py:87-106).

    The two computations are equal in exact arithmetic; they round differently: fake_quant rounds
    every dequantised operand q*s (+zp) to fp16 (relative 2^-11 each) and sums in fp32, the kernel
    path forms the exact integer dot product, rounds sa*sb to fp16 and the output to fp16. Bar:
      norm-wise  ||out - C_fq|| <= 1e-3 ||C_fq||            (north_star's 1e-3 relative)
      elementwise |out - C_fq| <= 1e-3 |C_fq| + 4e-3 rms(C_fq)   (cancellation floor)
    Measured on the fixtures: norm-wise 2-5e-4, elementwise excess <= 1.9e-3 rms."""
    out = out.astype(np.float64)
    ref = ref_fq.astype(np.float64)
    assert out.shape == ref.shape, (out.shape, ref.shape)
    if ref.size == 0:
        return
    assert np.isfinite(out).all(), f"{what}: non-finite output"
    nref = float(np.linalg.norm(ref))
    assert float(np.linalg.norm(out - ref)) <= 1e-3 * nref, f"{what}: norm-wise error above 1e-3"
    rms = nref / np.sqrt(ref.size)
    bad = np.abs(out - ref) > 1e-3 * np.abs(ref) + 4e-3 * rms
    assert not bad.any(), f"{what}: {bad.sum()} / {bad.size} outputs outside the fake-quant tolerance"


def codes_f64(packed: torch.Tensor, rows: int, bits: int, K: int) -> torch.Tensor:
    """pack_wxax rows -> their integer codes as f64 [rows, K]. The codes come out in the packed byte /
    nibble order (pack_wxax puts element 0 of each 16-bit word in its high bits, oracle/gg_oracle.c
    unpack_row), the same permutation of K for A and B, which leaves every dot product unchanged."""
    b = packed.contiguous().view(torch.int8).view(rows, -1)[:, :K * bits // 8]
    if bits == 8:
        return b.double()
    lo = torch.bitwise_right_shift(torch.bitwise_left_shift(b, 4), 4)  # sign-extended low nibble
    hi = torch.bitwise_right_shift(b, 4)                               # (arithmetic shift)
    return torch.stack((lo, hi), dim=-1).view(rows, -1).double()


def quant_epilogue_ref(acc, sa, sb):
    """oracle_gg_quant's epilogue on a whole f64 accumulator matrix (torch, any device):
    fp16_rn(0 + f32(acc) * f32(fp16_rn(sa[m] * sb[n]))) — the fp16 product of two fp16 scales is
    exact in f32 and rounded once, f32(acc) and the f32 product round to nearest, +0 turns -0 into +0."""
    s16 = sa.view(-1, 1).half() * sb.view(1, -1).half()
    return (acc.float() * s16.float() + 0.0).half()
