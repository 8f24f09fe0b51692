"""Bench harness — the Python restatement of the reference's C++ harness (src/test.cu, test_utils.h).

Reference behaviour mirrored:
  * inputs: uniform(-1, 1) fp16 A/B per problem, seeded (test.cu:877-915: default_random_engine(42));
    quantised problems are RTN-quantised per row and packed (QInput::from_fp16, test.cu:218-413) —
    unlike the reference bench (test.cu:518-521), the packed ints really are the quantised values
  * FLOPs = sum 2*M*N*K; TFLOPS = FLOPs / median_ms * 1e3 / 1e12 (test.cu:116, 154)
  * timing: up to 30 warmups, 50 timed iterations, median (test_utils.h:97-191)
  * CSV: kernel_name,avg_time,TFLOPS,speedup (test.cu:855-865)
Inputs are generated on the GPU (torch) so bs=8192 layers build in seconds; this is setup, not the
hot path.
"""
from __future__ import annotations

import csv
import dataclasses
import os
import statistics
from typing import Optional, Sequence

import torch

from .groupgemm import GroupGemm, Problem, QParams
from .quantize import pack_e4m3, pack_weightonly_mi355x, pack_wxax, quant_e4m3, quant_rtn_sym, quant_weightonly
from .workload import QShape


@dataclasses.dataclass
class LayerInputs:
    problems: list[Problem]
    shapes: list[QShape]

    @property
    def flops(self) -> int:
        return sum(s.flops for s in self.shapes)

    def bytes_algorithmic(self) -> int:
        """Packed A + packed B + fp16 C + fp16 scales."""
        tot = 0
        for s in self.shapes:
            plain = s.qcfg in ("fp16", "bf16")
            ab = 16 if plain else s.a_bits
            wb = 16 if plain else s.w_bits
            tot += (s.M * s.K * ab + s.N * s.K * wb) // 8 + 2 * s.M * s.N
            if not plain and ab == 16:  # weight-only: scale (+ zp) per column and group
                tot += 2 * s.N * (1 if s.gsize == -1 else s.K // s.gsize) * (1 if s.sym else 2)
            elif not plain:
                tot += 2 * (s.M + s.N) * (1 if s.gsize == -1 else s.K // s.gsize)
        return tot


def build_layer_inputs(shapes: Sequence[QShape], device="cuda", seed: int = 42,
                       out: Optional[torch.Tensor] = None) -> LayerInputs:
    """Allocate + fill one GroupGEMM call's inputs on `device` (one generator, problem order)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev).manual_seed(seed)
    probs = []
    for s in shapes:
        M, N, K = s.M, s.N, s.K
        q = QParams(a_bits=s.a_bits, w_bits=s.w_bits, gsize=s.gsize, sym=s.sym, fmt=s.fmt)
        a = (torch.rand(M, K, generator=g, device=dev) * 2 - 1).to(torch.float16)
        b = (torch.rand(N, K, generator=g, device=dev) * 2 - 1).to(torch.float16)
        C = torch.empty(max(M, 1), N, dtype=torch.float16, device=dev)
        if q.is_fp8:
            qa, sa = quant_e4m3(a)
            qb, sb = quant_e4m3(b)
            probs.append(Problem(A=pack_e4m3(qa), B=pack_e4m3(qb), C=C, M=M, N=N, K=K, q=q, scale_a=sa, scale_b=sb))
            del qa, qb
        elif q.fmt == "bf16":
            probs.append(Problem(A=a.to(torch.bfloat16), B=b.to(torch.bfloat16), C=C, M=M, N=N, K=K, q=q))
        elif q.is_weight_only:
            codes, sz = quant_weightonly(b, q.w_bits, q.gsize, q.sym)
            probs.append(Problem(A=a, B=pack_weightonly_mi355x(codes, q.w_bits), C=C, M=M, N=N, K=K, q=q,
                                 scale_b=sz))
            del codes
        elif q.is_quant:
            qa, sa = quant_rtn_sym(a, q.a_bits, q.gsize)
            qb, sb = quant_rtn_sym(b, q.w_bits, q.gsize)
            A, B = pack_wxax(qa, q.a_bits), pack_wxax(qb, q.w_bits)
            del qa, qb
            probs.append(Problem(A=A, B=B, C=C, M=M, N=N, K=K, q=q, scale_a=sa, scale_b=sb))
        else:
            probs.append(Problem(A=a, B=b, C=C, M=M, N=N, K=K, q=q))
        del a, b
    return LayerInputs(problems=probs, shapes=list(shapes))


class F6Layer:
    """A w4a4 call run on fp6 images (MXMOE_GG_FMT_F6, gg_f6.h): the B images are made once (weight
    preparation, as a serving stack keeps prepared weights), the A rows of every problem sit in one
    packed int4 buffer per K (as the MoE quantiser writes one permuted activation buffer) and
    ``pack_a()`` rebuilds their images — one mxmoe_gg_pack_f6 launch per distinct K, on the current
    stream — before each GEMM. ``problems`` read the images; results equal the int4 call's bit for bit."""

    def __init__(self, inputs: "LayerInputs"):
        from . import _native as nat
        from .groupgemm import W4A4_F6

        self.shapes = inputs.shapes
        ps = inputs.problems
        if any(p.q.qcfg != "w4a4_g-1_sym" for p in ps):
            raise ValueError("F6Layer: every problem must be w4a4_g-1_sym")
        dev = ps[0].C.device if ps else torch.device("cuda")
        self.a_groups = []  # (int4 rows [R, K/2], K, images [R, f6_row_bytes(K)])
        row_of = {}
        for K in sorted({p.K for p in ps}):
            sel = [i for i, p in enumerate(ps) if p.K == K]
            a4 = torch.cat([ps[i].A.reshape(max(ps[i].M, 0), K // 2) for i in sel]) if sel else None
            img = torch.empty((a4.shape[0], nat.f6_row_bytes(K)), dtype=torch.uint8, device=dev)
            r = 0
            for i in sel:
                row_of[i] = (len(self.a_groups), r)
                r += ps[i].M
            self.a_groups.append((a4, K, img))
        self.problems = []
        for i, p in enumerate(ps):
            g, r = row_of[i]
            img = self.a_groups[g][2]
            self.problems.append(dataclasses.replace(p, q=W4A4_F6, A=img[r:r + p.M], B=nat.pack_f6(p.B.reshape(p.N, p.K // 2), p.K),
                                                     lda=0, ldb=0))
        self.pack_a()
        torch.cuda.current_stream(dev).synchronize()

    def pack_a(self) -> None:
        from . import _native as nat

        for a4, K, img in self.a_groups:
            if a4.shape[0]:
                nat.pack_f6(a4, K, out=img)

    @property
    def flops(self) -> int:
        return sum(s.flops for s in self.shapes)


def refill_layer_inputs(inp: LayerInputs, seed: int = 42) -> None:
    """Regenerate a call's operands (the same seeded values as build_layer_inputs) in place, so a
    plan made on the buffers stays valid: operands materialised after planning, as a serving loop
    plans once per shape and receives data per batch."""
    dev = inp.problems[0].C.device if inp.problems else torch.device("cuda")
    fresh = build_layer_inputs(inp.shapes, device=dev, seed=seed)
    for p, q in zip(inp.problems, fresh.problems):
        for name in ("A", "B", "scale_a", "scale_b"):
            dst, src = getattr(p, name), getattr(q, name)
            if dst is not None:
                dst.copy_(src)
    del fresh


def time_launches(fn, warmup: int = 20, iters: int = 50, stream: Optional[torch.cuda.Stream] = None) -> dict:
    """Per-call device time with events on the launch stream; median / mean / min in ms."""
    s = stream if stream is not None else torch.cuda.current_stream()
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) for a, b in ev]
    return {"median_ms": statistics.median(ts), "mean_ms": sum(ts) / len(ts), "min_ms": min(ts), "iters": iters}


def bench_call(inputs: LayerInputs, variant: Optional[int] = None, warmup: int = 20, iters: int = 50) -> dict:
    gg = GroupGemm(inputs.problems, variant=variant)
    t = time_launches(gg.launch, warmup, iters)
    t["tflops"] = inputs.flops / (t["median_ms"] * 1e-3) / 1e12
    t["tiles"] = gg.total_tiles
    return t


def write_csv(path: str, rows: list[dict]) -> None:
    """CSV in the reference bench schema (test.cu:855-865)."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel_name", "avg_time", "TFLOPS", "speedup"])
        for r in rows:
            w.writerow([r["kernel_name"], f"{r['avg_time']:.6f}", f"{r['TFLOPS']:.3f}", f"{r['speedup']:.3f}"])


def slice_scale_b(p: Problem, n0: int, n1: int) -> Optional[torch.Tensor]:
    """scale_b entries of columns [n0, n1) in the layout the kernel reads for an N' = n1 - n0 problem:
    per-channel [N] -> a view; grouped [G][N] (w4a4 g128, weight-only sym) and weight-only asym
    [G][N][2] -> a contiguous copy of the [:, n0:n1] block (the kernel reads G x N' entries)."""
    if p.scale_b is None:
        return None
    q = p.q
    G = 1 if q.gsize == -1 else p.K // q.gsize
    if G == 1 and not (q.is_weight_only and not q.sym):
        return p.scale_b[n0:n1]
    return p.scale_b.reshape(G, p.N, -1)[:, n0:n1].contiguous().reshape(-1)


def slice_problem(p: Problem, n0: int, n1: int) -> Problem:
    """Columns [n0, n1) of a problem: B rows n0..n1 (a view), C columns n0..n1 (strided view, row
    stride = the full problem's ldc), scale_b per slice_scale_b (a copy only for grouped layouts)."""
    return dataclasses.replace(p, B=p.B[n0:n1], C=p.C[:, n0:n1], N=n1 - n0, ldc=p.ldc or p.N,
                               scale_b=slice_scale_b(p, n0, n1))


def slice_rows(p: Problem, m0: int, m1: int, C: Optional[torch.Tensor] = None) -> Problem:
    """Rows [m0, m1) of a problem (tokens): A rows (a view), C rows (a view, or `C`), scale_a per
    row — per-channel [M] -> a view, grouped [G][M] (w4a4 g128) -> a contiguous copy of [:, m0:m1]."""
    sa = p.scale_a
    if sa is not None:
        G = 1 if p.q.gsize == -1 else p.K // p.q.gsize
        sa = sa[m0:m1] if G == 1 else sa.reshape(G, p.M)[:, m0:m1].contiguous().reshape(-1)
    return dataclasses.replace(p, A=p.A[m0:m1], C=p.C[m0:m1] if C is None else C, M=m1 - m0, scale_a=sa,
                               ldc=0 if C is not None else p.ldc)


def ep_scaling_sim(gate_up: LayerInputs, down: LayerInputs, worlds: Sequence[int] = (2, 4, 8), warmup: int = 5,
                   iters: int = 20, variant: Optional[int] = None, shared: bool = True) -> dict:
    """Compute-only strong scaling of one layer split by expert (dist.ep_layer_plan, the N > 1
    headline's plan), measured on ONE GPU: every rank's gate_up + down calls over its row items are
    timed as their own calls (ranks are independent GPUs); T_G = max over ranks, speedup = T_1 / T_G.
    The all-gather of the down outputs that follows on a node is listed as MB received per rank."""
    from .dist import (XGMI_LINK_GBS, ep_combine_plan, ep_layer_plan, ep_shard_elems, exchange_model,
                       link_gbs_for_speedup, synthetic_routing)

    def t_pair(gu, dn):
        ggs = [GroupGemm(x, variant=variant) for x in (gu, dn) if x]
        return time_launches(lambda: [g.launch() for g in ggs], warmup, iters)["median_ms"]

    t1 = t_pair(gate_up.problems, down.problems)
    out = {"t1_ms": round(t1, 4)}
    for G in worlds:
        plan = ep_layer_plan(gate_up.shapes, down.shapes, G, shared)
        rank_ms = [t_pair([slice_rows(gate_up.problems[w.problem], w.m0, w.m1) for w in items],
                          [slice_rows(down.problems[w.problem], w.m0, w.m1) for w in items]) if items else 0.0
                   for items in plan]
        tg = max(rank_ms)
        pad = max(ep_shard_elems(down.shapes, items) for items in plan)
        H = down.shapes[0].N
        cplan = None
        if shared and all(s.N == H for s in down.shapes):  # the token-owner exchange (synthetic routing)
            routing = synthetic_routing([s.M for s in down.shapes[:-1]], down.shapes[-1].M,
                                        max(1, -(-sum(s.M for s in down.shapes[:-1]) // max(1, down.shapes[-1].M))))
            cplan = ep_combine_plan(plan, down.shapes, routing)
        model = exchange_model(tg, G, pad, cplan, H)
        out[str(G)] = {"t_ms_max_rank": round(tg, 4), "speedup": round(t1 / tg, 3),
                       "rank_ms": [round(x, 4) for x in rank_ms],
                       "allgather_MB_per_rank": round(2 * pad * (G - 1) / 1e6, 1),
                       "modelled": {k: {**v, "speedup": round(t1 / v["step_ms"], 3)} for k, v in model.items()},
                       # the effective GB/s per xGMI link (and direction) each exchange needs for 3.5x (None:
                       # not reachable at any link rate); the model above assumes XGMI_LINK_GBS
                       "link_GBs_for_3p5x": link_gbs_for_speedup(t1, tg, G, pad, cplan, H),
                       "link_GBs_assumed": XGMI_LINK_GBS}
    return out


def strong_scaling_sim(inputs: LayerInputs, worlds: Sequence[int] = (2, 4, 8), warmup: int = 5,
                       iters: int = 20, variant: Optional[int] = None) -> dict:
    """Compute-only strong scaling of one GroupGEMM call, measured on ONE GPU:
    each rank's work list of dist.nslice_plan runs as its own planned call; ranks are independent
    GPUs, so T_G = max over ranks of that time and speedup = T_1 / T_G. The C all-gather that
    follows on a real node is reported separately as bytes per rank (not timed here)."""
    from .dist import nslice_plan, shard_bytes

    t1 = time_launches(GroupGemm(inputs.problems, variant=variant).launch, warmup, iters)["median_ms"]
    out = {"t1_ms": round(t1, 4)}
    for G in worlds:
        plan = nslice_plan(inputs.shapes, G)
        per_rank = []
        for work in plan:
            probs = [slice_problem(inputs.problems[w.problem], w.n0, w.n1) for w in work]
            per_rank.append(time_launches(GroupGemm(probs, variant=variant).launch, warmup, iters)["median_ms"]
                            if probs else 0.0)
        tg = max(per_rank)
        out[str(G)] = {"t_ms_max_rank": round(tg, 4), "speedup": round(t1 / tg, 3),
                       "rank_ms": [round(x, 4) for x in per_rank],
                       "allgather_MB_per_rank": round(2 * max(shard_bytes(inputs.shapes, w) for w in plan) / 1e6, 1)}
    return out


def time_reference_abi(inputs: LayerInputs, iters: int = 20) -> float:
    """Wall ms per call of the reference-compatible entry (groupgemm_mxmoe: device pointer arrays,
    per-call host planning + upload + launch, legacy stream) — the 'as-reference' number, comparable
    with the reference host API that rebuilds its prefix array every call (kernel_sketch.py:87-143)."""
    import time

    from .groupgemm import groupgemm_reference_abi

    dev = inputs.problems[0].C.device

    def ptrs(get):
        return torch.tensor([0 if get(p) is None else get(p).data_ptr() for p in inputs.problems],
                            dtype=torch.int64, device=dev)

    arrs = [ptrs(lambda p: p.A), ptrs(lambda p: p.B), ptrs(lambda p: p.scale_a), ptrs(lambda p: p.scale_b),
            ptrs(lambda p: p.C)]
    sizes = [(p.M, p.N, p.K) for p in inputs.problems]
    qs = [p.q for p in inputs.problems]

    def call():
        groupgemm_reference_abi(*arrs, sizes, qs)

    for _ in range(3):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        call()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters
