"""bench.py — GroupGEMM TFLOP/s + %roofline, qwen2_moe layer-11 (bs=8192), MI355X.

One "step" = one pass of the hot path over one batch: the layer's two fused GroupGEMM calls
(gate_up: 61 problems, down: 61 problems), inputs resident in HBM, tile tables planned once.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config fp16|w8a8|w4a4|mixed] [--variant V]
  (N > 1: launched by torch.distributed.run, one rank per GPU)

Multi-GPU (strong scaling, SURVEY.md §8e, north_star): with N ranks the SAME layer is split by
expert (dist.ep_layer_plan): routed experts by index (LPT on gate_up + down FLOPs), the shared expert
by token rows sized to even out the ranks; each rank runs gate_up and down for its share (the gate_up
output is the down call's input and stays on its rank) and the layer's outputs — every rank's down C,
packed into one shard — are all-gathered over RCCL / xGMI. value = the layer's FLOPs / max-over-ranks
time of K such steps. extras.strong_scaling carries T1, compute-only and step times and both
speedups; extras.strong_scaling_nslice the N-slice split that all-gathers both calls' C (gate_up
gather overlapped with down); extras.ep_weak_scaling the expert-parallel weak-scaling number
(N x 8192 tokens, no collective).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

# The reference's published GroupGEMM TFLOPS (RTX-4090, read off media/final-perf.png by eye, about
# +-5 %) — context only: BASELINE.json publishes no number, so vs_baseline stays null.
REFERENCE_CHART_TFLOPS = {"fp16": 145.0, "w8a8": 420.0, "w4a4": 690.0, "mixed": 545.0, "ds2_mixed": 578.0,
                          "w4a16_w8a8_bs512": 115.0}  # bs=512 W4.25A15.5 bar

PEAK_TFLOPS = {"fp16": 2500.0, "int8": 5000.0, "fp8": 5000.0}  # dense MFMA peaks, MI355X_MICROARCH.md (spec)
HBM_GBS = 8000.0

CONFIGS = {
    "fp16": dict(kw={}, peak="fp16", dtype="fp16", name="qwen2_moe layer-11 fp16 GroupGEMM bs=8192, 60 experts"),
    "w8a8": dict(kw=dict(qstr="w8a8_g-1_sym"), peak="int8", dtype="int8",
                 name="qwen2_moe layer-11 w8a8_g-1_sym GroupGEMM bs=8192 (int8 MFMA)"),
    "w4a4": dict(kw=dict(qstr="w4a4_g-1_sym"), peak="int8", dtype="int4",
                 name="qwen2_moe layer-11 w4a4_g-1_sym GroupGEMM bs=8192 (int8 MFMA)"),
    "mixed": dict(kw="mixed", peak="int8", dtype="int4+int8",
                  name="qwen2_moe layer-11 mixed w4a4+w8a8 (wbits=5.0, LP-1 qconfig) bs=8192"),
    "ds2_mixed": dict(kw="ds2_mixed", peak="int8", dtype="int4+int8",
                      name="DeepSeek-V2-Lite MoE layer mixed w4a4+w8a8 (25 % w8a8 units) bs=8192, 64 experts"),
    # w4a4 g128: int4 A / B, one scale per 128-K group, f32 fold per group
    "w4a4_g128": dict(kw=dict(qstr="w4a4_g128_sym"), peak="int8", dtype="int4 (g128)",
                      name="qwen2_moe layer-11 w4a4_g128_sym GroupGEMM bs=8192 (int8 MFMA + per-group f32 fold)"),
    # weight-only: fp16 activations, int4 weights dequantised to fp16 MFMA
    "w4a16": dict(kw=dict(qstr="w4a16_g128_asym"), peak="fp16", dtype="fp16 (int4 weights)",
                  name="qwen2_moe layer-11 w4a16_g128_asym GroupGEMM bs=8192"),
    "w4a16_bs512": dict(kw=dict(qstr="w4a16_g128_asym"), peak="fp16", dtype="fp16 (int4 weights)", bs=512,
                        name="qwen2_moe layer-11 w4a16_g128_asym GroupGEMM bs=512 (weight-bandwidth bound)"),
    "w2a16": dict(kw=dict(qstr="w2a16_g128_asym"), peak="fp16", dtype="fp16 (int2 weights)",
                  name="qwen2_moe layer-11 w2a16_g128_asym GroupGEMM bs=8192"),
    "w2a16_bs512": dict(kw=dict(qstr="w2a16_g128_asym"), peak="fp16", dtype="fp16 (int2 weights)", bs=512,
                        name="qwen2_moe layer-11 w2a16_g128_asym GroupGEMM bs=512 (weight-bandwidth bound)"),
    "fp16_bs512": dict(kw={}, peak="fp16", dtype="fp16", bs=512,
                       name="qwen2_moe layer-11 fp16 GroupGEMM bs=512"),
    # the reference's published small-batch mixed scheme (W4.25A15.5, README / SURVEY §6): w4a16_g-1_asym
    # + w8a8_g-1_sym per linear block in one fused launch (hz_fused.cuh:14-125, ref_bind.cu:412)
    "w4a16_w8a8_bs512": dict(kw="w4a16_w8a8", peak="fp16", dtype="fp16 (int4 weights) + int8", bs=512,
                             name="qwen2_moe layer-11 mixed w4a16_g-1_asym + w8a8_g-1_sym (W4.25A15.5) GroupGEMM "
                                  "bs=512 (weight-bandwidth bound)"),
    # the reference's other SUPPORTED_QCFG strategies (tile_config.py:40-106)
    "w8a8_e4m3": dict(kw=dict(qstr="w8a8_g-1_sym_E4M3"), peak="fp8", dtype="fp8 e4m3",
                      name="qwen2_moe layer-11 w8a8_g-1_sym_E4M3 GroupGEMM bs=8192 (fp8 MFMA, f32 accumulate)"),
    "bf16": dict(kw=dict(qstr="bf16"), peak="fp16", dtype="bf16",
                 name="qwen2_moe layer-11 bf16 GroupGEMM bs=8192"),
    # the reference CLI's other models (gen_workload.py:16-21), seeded synthetic routing
    "mixtral_fp16": dict(kw={}, model="mixtral", peak="fp16", dtype="fp16",
                         name="Mixtral-8x7B MoE layer fp16 GroupGEMM bs=8192 (8 experts, top-2)"),
    "mixtral_w8a8": dict(kw=dict(qstr="w8a8_g-1_sym"), model="mixtral", peak="int8", dtype="int8",
                         name="Mixtral-8x7B MoE layer w8a8_g-1_sym GroupGEMM bs=8192"),
    "qwen2_57b_fp16": dict(kw={}, model="qwen2_moe_57b", peak="fp16", dtype="fp16",
                           name="Qwen2-57B-A14B MoE layer fp16 GroupGEMM bs=8192 (64 experts, top-8, shared)"),
    "qwen2_57b_w8a8": dict(kw=dict(qstr="w8a8_g-1_sym"), model="qwen2_moe_57b", peak="int8", dtype="int8",
                           name="Qwen2-57B-A14B MoE layer w8a8_g-1_sym GroupGEMM bs=8192"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def layer_shapes(cfg: str, world: int, rank: int, bs: int = 8192):
    """Per-rank problem lists {gate_up, down} (expert-parallel weak scaling, mxmoe_amd/dist.py)."""
    from mxmoe_amd.dist import ep_shard

    return ep_shard(full_layer(cfg, bs), world, rank)


def full_layer(cfg: str, bs: int = 8192):
    """The config's whole layer {gate_up, down} (one GPU's worth at N = 1)."""
    from mxmoe_amd.workload import (ds2_mixed_qconfig, ds2_workload, load_workload, mixed_qconfig_lp1,
                                    model_workload, qwen2_layer11_workload)

    bs = CONFIGS[cfg].get("bs", bs)
    kw = CONFIGS[cfg]["kw"]
    if "model" in CONFIGS[cfg]:
        return load_workload(model_workload(CONFIGS[cfg]["model"], bs, **kw))["layer-1"]
    if kw == "ds2_mixed":
        return load_workload(ds2_workload(bs, qconfig=ds2_mixed_qconfig()))["layer-1"]
    if kw == "mixed":
        kw = dict(qconfig=mixed_qconfig_lp1())
    elif kw == "w4a16_w8a8":
        from mxmoe_amd.workload import w4a16_w8a8_qconfig

        kw = dict(qconfig=w4a16_w8a8_qconfig())
    return load_workload(qwen2_layer11_workload(bs, **kw))["layer-11"]


def strong_scaling_step(cfg: str, dev, world: int, rank: int, steps: int, warmup: int, coll_dev, variant=None,
                        median_iters: int = 50, settle_s: float = 0.0) -> dict:
    """The N > 1 headline (SURVEY.md §8e, strong scaling): ONE layer (the N = 1 workload) split over
    the ranks by dist.nslice_plan. Every rank holds the full inputs (same seeds), runs its work list
    with its C slices packed into one local shard, and the shards are all-gathered over RCCL / xGMI;
    the gate_up gather runs on a second stream while down computes (dist.ShardedLayerStep).
    Timed K steps between barriers + synchronisations, max over ranks, for: the full layer on one GPU
    (T1, every rank), the sharded compute only, and compute + all-gathers (the step)."""
    import torch.distributed as dist

    from mxmoe_amd.dist import ShardedCall, ShardedLayerStep
    from mxmoe_amd.groupgemm import GroupGemm
    from mxmoe_amd.harness import build_layer_inputs, time_launches

    layer = full_layer(cfg)
    inp = {gg: build_layer_inputs(layer[gg], device=dev, seed=42 + (gg == "down")) for gg in ("gate_up", "down")}
    stream = torch.cuda.current_stream(dev)

    def timed(fn, k=steps, w=warmup, settle=0.0):
        # settle: seconds of untimed calls first — only for a collective-free fn (the count of calls
        # may differ between ranks)
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < settle:
            for _ in range(4):
                fn()
            torch.cuda.synchronize(dev)
        for _ in range(w):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    full = {gg: GroupGemm(inp[gg].problems, variant=variant, device=dev) for gg in inp}
    t1 = timed(lambda: (full["gate_up"].launch(stream), full["down"].launch(stream)), settle=settle_s)
    del full
    calls = {gg: ShardedCall(inp[gg], world, rank, variant=variant) for gg in inp}
    step = ShardedLayerStep(calls["gate_up"], calls["down"], overlap=True)
    serial = ShardedLayerStep(calls["gate_up"], calls["down"], overlap=False)
    t_comp = timed(lambda: step.compute_only(stream))
    t_serial = timed(lambda: serial(stream))
    t_step = timed(lambda: step(stream))
    flops = float(inp["gate_up"].flops + inp["down"].flops)
    per = {gg: (time_launches(lambda g=gg: calls[g].compute(stream), warmup=3, iters=median_iters, stream=stream)
                if calls[gg].part is not None else {"mean_ms": 0.0, "median_ms": 0.0}) for gg in calls}
    return {"dt": t_step, "total_flops": flops, "t1": t1, "t_compute": t_comp, "t_serial": t_serial,
            "per": per, "flops_local": {gg: calls[gg].flops_local for gg in calls},
            "bytes_local": {gg: sum(calls[gg].shapes[w.problem].M * w.width * 2 +
                                    (calls[gg].shapes[w.problem].M + w.width) * calls[gg].shapes[w.problem].K *
                                    (16 if calls[gg].shapes[w.problem].qcfg == "fp16" else calls[gg].shapes[w.problem].a_bits) // 8
                                    for w in calls[gg].plan[rank]) for gg in calls},
            "allgather_MB_per_rank": {gg: round(2 * calls[gg].pad * (world - 1) / 1e6, 1) for gg in calls},
            "variant": calls["gate_up"].part.variant if calls["gate_up"].part is not None else -1,
            "tiles": {gg: calls[gg].part.total_tiles if calls[gg].part is not None else 0 for gg in calls}}


def _gather_only(step, stream) -> None:
    with torch.cuda.stream(stream):
        step.gather()


def ep_layer_step(cfg: str, dev, world: int, rank: int, steps: int, warmup: int, coll_dev, variant=None,
                  median_iters: int = 50, settle_s: float = 0.0) -> dict:
    """The N > 1 headline: ONE layer (the N = 1 workload) split by expert over the ranks
    (dist.EPLayerStep). Every rank holds the full inputs (same seeds), runs gate_up and down over its
    row items, and the packed down outputs are all-gathered over RCCL / xGMI. Timed K steps between
    barriers + synchronisations, max over ranks, for: the full layer on one GPU (T1, every rank), the
    sharded compute only, and compute + all-gather (the step)."""
    import torch.distributed as dist

    from mxmoe_amd.dist import EPLayerStep, choose_chunks, gather_ms_model
    from mxmoe_amd.groupgemm import GroupGemm
    from mxmoe_amd.harness import build_layer_inputs, time_launches

    layer = full_layer(cfg)
    inp = {gg: build_layer_inputs(layer[gg], device=dev, seed=42 + (gg == "down")) for gg in ("gate_up", "down")}
    stream = torch.cuda.current_stream(dev)

    def timed(fn, k=steps, w=warmup, settle=0.0):
        # settle: seconds of untimed calls first — only for a collective-free fn (the count of calls
        # may differ between ranks)
        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < settle:
            for _ in range(4):
                fn()
            torch.cuda.synchronize(dev)
        for _ in range(w):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    full = {gg: GroupGemm(inp[gg].problems, variant=variant, device=dev) for gg in inp}
    t1 = timed(lambda: (full["gate_up"].launch(stream), full["down"].launch(stream)), settle=settle_s)
    del full
    shared = CONFIGS[cfg].get("model") != "mixtral"
    step = EPLayerStep(inp["gate_up"], inp["down"], world, rank, variant=variant, shared=shared)
    t_comp = timed(lambda: step.compute(stream))
    t_gather = timed(lambda: _gather_only(step, stream))
    t_step = timed(lambda: step(stream))
    # the compute / all-gather pipeline depth: dist.choose_chunks on this node's measured compute and
    # gather times (max over ranks), then the chosen split timed as the headline step
    chunks = choose_chunks(t_comp / steps * 1e3, t_gather / steps * 1e3)
    if chunks > 1:
        stepc = EPLayerStep(inp["gate_up"], inp["down"], world, rank, variant=variant, shared=shared, chunks=chunks)
        t_stepc = timed(lambda: stepc(stream))
        t_compc = timed(lambda: stepc.compute(stream))
        del stepc
    else:
        t_stepc, t_compc = t_step, t_comp
    flops = float(inp["gate_up"].flops + inp["down"].flops)
    none = {"mean_ms": 0.0, "median_ms": 0.0}
    per = {"gate_up": time_launches(lambda: step.gu.launch(stream), warmup=3, iters=median_iters, stream=stream)
           if step.gu is not None else none,
           "down": time_launches(lambda: step.dn.launch(stream), warmup=3, iters=median_iters, stream=stream)
           if step.dn is not None else none}

    def nbytes(shapes, w):
        s = shapes[w.problem]
        bits_a = 16 if s.a_bits == 16 else s.a_bits
        return w.rows * s.N * 2 + w.rows * s.K * bits_a // 8 + s.N * s.K * s.w_bits // 8

    mine = step.plan[rank]
    gg_of = {"gate_up": step.gu, "down": step.dn}
    return {"dt": t_stepc, "total_flops": flops, "t1": t1, "t_compute": t_comp, "per": per,
            "chunks": chunks, "t_step_1chunk": t_step, "t_compute_chunked": t_compc, "t_gather": t_gather,
            "gather_model_ms": gather_ms_model(2 * step.pad * (world - 1), world),
            "flops_local": step.flops_local,
            "bytes_local": {"gate_up": sum(nbytes(step.shapes_gu, w) for w in mine),
                            "down": sum(nbytes(step.shapes_dn, w) for w in mine)},
            "allgather_MB_received_per_rank": round(2 * step.pad * (world - 1) / 1e6, 1),
            "items": len(mine),
            "variant": (step.gu or step.dn).variant if (step.gu or step.dn) is not None else -1,
            "tiles": {gg: g.total_tiles if g is not None else 0 for gg, g in gg_of.items()}}


def ep_combine_step(cfg: str, dev, world: int, rank: int, steps: int, warmup: int, coll_dev, variant=None) -> dict:
    """The second N > 1 step (dist.EPCombineStep): the same expert split and compute as ep_layer_step,
    then the token-owner exchange — routed down rows all-to-all'ed to their token's owner, combined
    there in top-k order with its shared-expert rows (HIP mxmoe_moe_combine), the combined [T, H]
    output all-gathered — instead of all-gathering every expert's down C. Synthetic routing consistent
    with the workload's per-expert rows (dist.synthetic_routing)."""
    import torch.distributed as dist

    from mxmoe_amd.dist import EPCombineStep, synthetic_routing
    from mxmoe_amd.harness import build_layer_inputs

    layer = full_layer(cfg)
    inp = {gg: build_layer_inputs(layer[gg], device=dev, seed=42 + (gg == "down")) for gg in ("gate_up", "down")}
    dn = layer["down"]
    T = dn[-1].M
    topk = -(-sum(s.M for s in dn[:-1]) // T)
    step = EPCombineStep(inp["gate_up"], inp["down"], world, rank, synthetic_routing([s.M for s in dn[:-1]], T, topk),
                         variant=variant)
    stream = torch.cuda.current_stream(dev)

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        dist.barrier()
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    t_comp = timed(lambda: step.compute(stream))
    t_x = timed(lambda: step.exchange(stream))
    t_step = timed(lambda: step(stream))
    b = step.cplan.bytes_received(dn[0].N)
    return {"t_compute": t_comp, "t_exchange": t_x, "dt": t_step, "topk": topk,
            "a2a_MB_received_max": round(max(b["all_to_all"]) / 1e6, 1),
            "allgather_out_MB_received": round(max(b["allgather_out"]) / 1e6, 1)}


def cpu_info() -> dict:
    """Host CPU model and the threads the baseline may use (the GPU box exports OMP_NUM_THREADS=16:
    its share of a much larger machine, which os.cpu_count() would report)."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = min(avail, int(os.environ.get("OMP_NUM_THREADS", avail)))
    return {"model": model, "threads": max(1, threads), "visible_cpus": avail}


def cpu_baseline(cfg: str, shapes, budget_s: float = 12.0) -> dict:
    """The reference's torch CPU matmul path, timed on this host's cores on a bounded
    sample of the same layer: one torch.matmul(A_i, B_i.T) per problem — fp16 operands for fp16
    problems; int-valued fp32 operands plus the reference epilogue
    fp16(f32(acc) * f32(fp16(sa * sb))) (mm_tile.cuh:469-496) for quantised ones. Routed problems of
    gate_up then down in call order until ~budget_s / 3 of CPU time, then 1 warm-up + 3 timed passes
    over that sample. A reported baseline, not the optimisation target."""
    info = cpu_info()
    torch.set_num_threads(info["threads"])
    g = torch.Generator().manual_seed(0)
    sample, est = [], 0.0
    for gg in ("gate_up", "down"):
        for sh in shapes[gg][:-1]:
            if sh.M == 0:
                continue
            if sh.qcfg in ("fp16", "bf16"):
                dt = torch.bfloat16 if sh.qcfg == "bf16" else torch.float16
                a = (torch.rand(sh.M, sh.K, generator=g) * 2 - 1).to(dt)
                b = (torch.rand(sh.N, sh.K, generator=g) * 2 - 1).to(dt)
                sa = sb = None
            elif sh.fmt == "E4M3":  # decoded fp8 values as fp32 operands (exact), then the epilogue
                a = (torch.rand(sh.M, sh.K, generator=g) * 2 - 1).mul(448).to(torch.float8_e4m3fn).float()
                b = (torch.rand(sh.N, sh.K, generator=g) * 2 - 1).mul(448).to(torch.float8_e4m3fn).float()
                sa = (torch.rand(sh.M, generator=g) * 0.01).half()
                sb = (torch.rand(sh.N, generator=g) * 0.01).half()
            else:
                qm = (1 << (sh.a_bits - 1)) - 1
                a = torch.randint(-qm, qm + 1, (sh.M, sh.K), generator=g).float()
                b = torch.randint(-qm, qm + 1, (sh.N, sh.K), generator=g).float()
                sa = (torch.rand(sh.M, generator=g) * 0.01).half()
                sb = (torch.rand(sh.N, generator=g) * 0.01).half()
            sample.append((gg, sh, a, b, sa, sb))
            t0 = time.perf_counter()
            one_problem(a, b, sa, sb)
            est += time.perf_counter() - t0
            if est > budget_s / 3:
                break
        if est > budget_s / 3:
            break

    def run_pass():
        for _, _, a, b, sa, sb in sample:
            one_problem(a, b, sa, sb)

    run_pass()  # warm-up
    t0 = time.perf_counter()
    for _ in range(3):
        run_pass()
    dt = (time.perf_counter() - t0) / 3
    flops = sum(2 * sh.M * sh.N * sh.K for _, sh, *_ in sample)
    names = [f"{gg}[{sh.M}x{sh.N}x{sh.K} {sh.qcfg}]" for gg, sh, *_ in sample]
    shown = ", ".join(names[:3]) + (f", ... ({len(names) - 3} more)" if len(names) > 3 else "")
    return {"value": round(flops / dt / 1e12, 6), "unit": "TFLOP/s", "cores": info["threads"], "kind": "port",
            "impl": "torch.matmul(A_i, B_i.T) per problem on the host (the reference's torch CPU matmul path); "
                    + {"fp16": "fp16 operands", "bf16": "bf16 operands",
                       "w8a8_e4m3": "decoded e4m3 values as fp32 operands + fp16 scale epilogue"}.get(
                        cfg.split("_", 1)[1] if cfg.startswith(("mixtral_", "qwen2_57b_")) else cfg,
                        "int-valued fp32 operands + fp16 scale epilogue"),
            "cpu_model": info["model"], "threads": info["threads"], "visible_cpus": info["visible_cpus"],
            "sample": f"{len(sample)} routed-expert problems of the same layer in call order ({shown}); "
                      f"{flops / 1e9:.1f} GFLOP per pass, 1 warm-up + 3 timed passes, {dt * 1e3:.0f} ms per pass"}


def one_problem(a, b, sa, sb):
    """One problem of the CPU baseline: C = A . B^T (+ the quantised epilogue)."""
    acc = torch.matmul(a, b.t())
    if sa is None:
        return acc
    s16 = (sa.float()[:, None] * sb.float()[None, :]).half().float()
    return (acc * s16).half()


def load_pmc_traffic(cfg: str):
    """The committed counter bytes of `cfg` (profiles/pmc_traffic.json, tools/pmc_traffic.sh), with
    `_source`: which round's tree measured them (the file's `_round` / per-config `_round` tags)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
        c = d.get(cfg)
        if isinstance(c, dict):
            rnd = c.get("_round", d.get("_round", "unknown round"))
            c = {**c, "_source": f"profiles/pmc_traffic.json ({rnd}; FETCH_SIZE x2 + WRITE_SIZE per step)"}
        return c
    except Exception:  # pragma: no cover
        return None


def resolve_launch(gpus: int, env, device_count: int) -> tuple[str, str]:
    """What `bench.py --gpus N` does in this process: ("run", "") runs the ranks' code here (N = 1, or
    one rank of a launcher that set WORLD_SIZE = N), ("spawn", "") starts N rank processes through
    torch.distributed.run as a child, ("error", why) refuses. Decided before any GPU call: counting
    devices does not initialise the GPU on this image. The one-GPU sharing of several ranks is a gloo
    rehearsal only (MXMOE_DIST_BACKEND=gloo and MXMOE_DIST_SHARE_GPU=1); under RCCL every rank needs a
    GPU of its own."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    backend = env.get("MXMOE_DIST_BACKEND", "nccl")
    share = backend == "gloo" and env.get("MXMOE_DIST_SHARE_GPU", "0") == "1"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", f"WORLD_SIZE={world} but --gpus {gpus}: n_gpus must equal --gpus"
        if world > 1 and device_count < world and not share:
            return "error", (f"{world} ranks but {device_count} visible GPU(s); ranks never share a GPU under "
                             f"{backend} (set MXMOE_DIST_BACKEND=gloo MXMOE_DIST_SHARE_GPU=1 to rehearse on one GPU)")
        return "run", ""
    if gpus == 1:
        return "run", ""
    if device_count < gpus and not share:
        return "error", (f"--gpus {gpus} but {device_count} visible GPU(s) (set MXMOE_DIST_BACKEND=gloo "
                         f"MXMOE_DIST_SHARE_GPU=1 to rehearse on one GPU)")
    return "spawn", ""


def spawn_ranks(gpus: int, argv: list[str]) -> list[str]:
    """The torch.distributed.run command that starts `gpus` ranks of this script with the same
    arguments (run as a child process: this process never touches the GPU, so no exec is needed)."""
    import socket

    with socket.socket() as s:  # a free port on the loopback rendezvous address
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # the chip needs ~0.2 s of sustained load to reach its steady clock: 10 warm-up steps read 3-5 %
    # low on the headline and 5-8 % on the extras (profiles/r02/verify2/warmup_ab.jsonl)
    ap.add_argument("--warmup", type=int, default=200)
    # clock settle before the W warm-up steps: the timed steps then run at the steady clock whatever W
    # the caller picks (round 3's driver run used W = 5: 0.398 of peak on the step clock against
    # 0.436 on the kernels' own clock)
    ap.add_argument("--settle-s", type=float, default=0.3, help="seconds of untimed steps before the warm-up")
    ap.add_argument("--config", default="fp16", choices=list(CONFIGS))
    ap.add_argument("--no-scaling-sim", action="store_true",
                    help="skip the single-GPU strong-scaling simulation and the as-reference timing (N=1 only)")
    ap.add_argument("--variant", type=int, default=-1, help="-1 = library's choice (MXMOE_GG_VARIANT_AUTO)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-moe-layer", action="store_true",
                    help="skip extras.moe_layer (the qwen2_moe layer-11 MoE FFN step, unfused vs fused SiLU epilogue)")
    ap.add_argument("--dist-extras-all", action="store_true",
                    help="N > 1: also run the N-slice strong-scaling and EP weak-scaling extras (off by default: "
                         "the default N > 1 run exercises one RCCL path, the expert split)")
    ap.add_argument("--extras", default="w8a8,w4a4,mixed,ds2_mixed,w4a16_w8a8_bs512,w4a16_bs512", help="other configs measured as extra fields (N=1)")
    ap.add_argument("--median-iters", type=int, default=50)
    ap.add_argument("--materialise-after-plan", action=argparse.BooleanOptionalAction, default=True,
                    help="N = 1: plan the two calls on the allocated buffers, then (re)generate the operands, "
                         "so the host planning does not sit between the data and the launches")
    ap.add_argument("--dist-extras", default="ds2_mixed", help="other configs run through the expert split at N > 1")
    ap.add_argument("--extras-warmup", type=int, default=200, help="untimed steps before an extra config's launch timing")
    args = ap.parse_args()

    action, why = resolve_launch(args.gpus, os.environ, torch.cuda.device_count())
    if action == "error":
        log("bench.py: " + why)
        sys.exit(2)
    if action == "spawn":
        import subprocess

        sys.exit(subprocess.call(spawn_ranks(args.gpus, sys.argv[1:])))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MXMOE_DIST_BACKEND=gloo rehearses the N > 1 path (collectives staged through host memory; with
    # MXMOE_DIST_SHARE_GPU=1 several ranks may share one GPU); the node runs use RCCL ("nccl")
    backend = os.environ.get("MXMOE_DIST_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist

        if local >= torch.cuda.device_count():  # resolve_launch allowed it: the gloo one-GPU rehearsal
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")  # where small collective tensors live

    from mxmoe_amd import _native as nat
    from mxmoe_amd.groupgemm import GroupGemm
    from mxmoe_amd.harness import build_layer_inputs, refill_layer_inputs, time_launches

    def run_config(cfg: str, steps: int, warmup: int, timed_region: bool):
        variant = args.variant if args.variant >= 0 else None
        shapes = layer_shapes(cfg, world, rank)
        inp = {gg: build_layer_inputs(shapes[gg], device=dev, seed=42 + 1000 * rank + (gg == "down"))
               for gg in ("gate_up", "down")}
        ggs = {gg: GroupGemm(inp[gg].problems, variant=variant, device=dev) for gg in inp}
        variant = ggs["gate_up"].variant  # concrete (AUTO resolved by the library)
        if args.materialise_after_plan:  # plan once per shape, then the batch's data (a serving loop's order)
            for gg in ("gate_up", "down"):
                refill_layer_inputs(inp[gg], seed=42 + 1000 * rank + (gg == "down"))
        flops = {gg: inp[gg].flops for gg in inp}
        stream = torch.cuda.current_stream(dev)

        def step():
            ggs["gate_up"].launch(stream)
            ggs["down"].launch(stream)

        t_settle = time.perf_counter()
        while time.perf_counter() - t_settle < args.settle_s:
            for _ in range(4):
                step()
            torch.cuda.synchronize(dev)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        res = {}
        if timed_region:
            if world > 1:
                torch.distributed.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            if world > 1:
                torch.distributed.barrier()
                t = torch.tensor([dt], device=coll_dev, dtype=torch.float64)
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
                dt = float(t.item())
                f = torch.tensor([float(flops["gate_up"] + flops["down"])], device=coll_dev, dtype=torch.float64)
                torch.distributed.all_reduce(f)
                total_flops = float(f.item())
            else:
                total_flops = float(flops["gate_up"] + flops["down"])
            res["dt"] = dt
            res["total_flops"] = total_flops
        # per-launch device time (HIP events on the launch stream) — the roofline's denominator
        per = {gg: time_launches(lambda g=gg: ggs[g].launch(stream), warmup=3, iters=args.median_iters, stream=stream)
               for gg in ggs}
        res.update(per=per, flops=flops, variant=variant, tiles={gg: ggs[gg].total_tiles for gg in ggs},
                   bytes={gg: inp[gg].bytes_algorithmic() for gg in inp}, shapes=shapes)
        del ggs, inp
        torch.cuda.empty_cache()
        return res

    cfg = args.config
    peak = PEAK_TFLOPS[CONFIGS[cfg]["peak"]]
    extras = {}
    if world == 1:
        main_res = run_config(cfg, args.steps, args.warmup, True)
        f_gu, f_dn = main_res["flops"]["gate_up"], main_res["flops"]["down"]
        b_step = main_res["bytes"]["gate_up"] + main_res["bytes"]["down"]
    else:
        # strong scaling of ONE layer over the node, split by expert (north_star): value = the
        # layer's FLOPs / max-rank time of compute + the RCCL all-gather of the layer's outputs
        vv = args.variant if args.variant >= 0 else None
        eres = ep_layer_step(cfg, dev, world, rank, args.steps, args.warmup, coll_dev, variant=vv,
                             median_iters=args.median_iters, settle_s=args.settle_s)
        main_res = {"dt": eres["dt"], "total_flops": eres["total_flops"], "per": eres["per"],
                    "flops": eres["flops_local"], "variant": eres["variant"], "tiles": eres["tiles"],
                    "shapes": full_layer(cfg)}
        f_gu, f_dn = eres["flops_local"]["gate_up"], eres["flops_local"]["down"]
        b_step = eres["bytes_local"]["gate_up"] + eres["bytes_local"]["down"]
        ms = lambda t: t / args.steps * 1e3  # noqa: E731
        extras["strong_scaling"] = {
            "what": "one layer split by expert (dist.ep_layer_plan: routed experts by index, shared expert by token "
                    "rows); T1 = the whole layer on one GPU (max over ranks), compute = max-rank time of the local "
                    "gate_up + down calls, gather = the all_gather_into_tensor (RCCL on a node) of the packed down outputs "
                    "alone, step (value) = compute and gather pipelined in `chunks` chunks (dist.choose_chunks on "
                    "the measured compute / gather times), step_1chunk = compute then gather",
            "t1_ms": round(ms(eres["t1"]), 4), "compute_ms": round(ms(eres["t_compute"]), 4),
            "gather_ms": round(ms(eres["t_gather"]), 4), "gather_model_ms": round(eres["gather_model_ms"], 4),
            "chunks": eres["chunks"], "step_ms": round(ms(eres["dt"]), 4),
            "step_1chunk_ms": round(ms(eres["t_step_1chunk"]), 4),
            "compute_chunked_ms": round(ms(eres["t_compute_chunked"]), 4),
            "speedup_compute": round(eres["t1"] / eres["t_compute"], 3),
            "speedup_with_allgather": round(eres["t1"] / eres["dt"], 3),
            "allgather_MB_received_per_rank": eres["allgather_MB_received_per_rank"]}
        try:  # the token-owner exchange (combine before the exchange): VERDICT r04 item 6
            cres = ep_combine_step(cfg, dev, world, rank, args.steps, args.warmup, coll_dev, variant=vv)
            extras["strong_scaling"]["combine_exchange"] = {
                "what": "same split and compute; routed down rows all_to_all_single'd to their token's owner (the "
                        "rank holding that token's shared-expert rows), combined there (mxmoe_moe_combine, top-k "
                        "order), the combined [T, hidden] output all-gathered (dist.EPCombineStep)",
                "compute_ms": round(ms(cres["t_compute"]), 4), "exchange_ms": round(ms(cres["t_exchange"]), 4),
                "step_ms": round(ms(cres["dt"]), 4), "speedup_with_exchange": round(eres["t1"] / cres["dt"], 3),
                "a2a_MB_received_max": cres["a2a_MB_received_max"],
                "allgather_out_MB_received": cres["allgather_out_MB_received"]}
        except Exception as e:  # an extra must not lose the headline
            extras["strong_scaling"]["combine_exchange"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        for x in [e for e in args.dist_extras.split(",") if e and e != cfg]:
            try:  # BASELINE configs[4]: DeepSeek-V2-Lite mixed w4a4+w8a8 split by expert over the node
                xr = ep_layer_step(x, dev, world, rank, args.steps, args.warmup, coll_dev, variant=vv,
                                   median_iters=10)
                extras[x + "_ep"] = {
                    "what": CONFIGS[x]["name"] + f", one layer split by expert over {world} GPUs + "
                                                 f"{'RCCL' if backend == 'nccl' else backend} all-gather of the layer outputs",
                    "tflops": round(xr["total_flops"] * args.steps / xr["dt"] / 1e12, 3),
                    "step_ms": round(ms(xr["dt"]), 4), "t1_ms": round(ms(xr["t1"]), 4),
                    "compute_ms": round(ms(xr["t_compute"]), 4),
                    "speedup_compute": round(xr["t1"] / xr["t_compute"], 3),
                    "speedup_with_allgather": round(xr["t1"] / xr["dt"], 3), "chunks": xr["chunks"]}
            except Exception as e:  # an extra must not lose the headline
                extras[x + "_ep"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if args.dist_extras_all:
            try:  # the N-slice split: both calls' C all-gathered (gate_up gather beside down)
                sres = strong_scaling_step(cfg, dev, world, rank, args.steps, args.warmup, coll_dev, variant=vv,
                                           median_iters=10, settle_s=args.settle_s)
                extras["strong_scaling_nslice"] = {
                    "what": "one layer split by dist.nslice_plan; step = compute + all-gather of every call's C "
                            "(gate_up gather on a second stream beside the down call), serial = without the overlap",
                    "step_ms": round(ms(sres["dt"]), 4), "compute_ms": round(ms(sres["t_compute"]), 4),
                    "serial_ms": round(ms(sres["t_serial"]), 4),
                    "speedup_with_allgather": round(sres["t1"] / sres["dt"], 3),
                    "allgather_MB_received_per_rank": sres["allgather_MB_per_rank"]}
            except Exception as e:  # an extra must not lose the headline
                extras["strong_scaling_nslice"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if args.dist_extras_all:
            try:  # the round-1 headline, kept as an extra: expert-parallel weak scaling, no collective
                ep = run_config(cfg, args.steps, args.warmup, True)
                extras["ep_weak_scaling"] = {
                    "what": "global batch N x 8192 tokens, routed experts sharded by index (LPT), shared expert "
                            "replicated on local tokens; no collective (dispatch / combine is MoE plumbing)",
                    "value_tflops": round(ep["total_flops"] * args.steps / ep["dt"] / 1e12, 3),
                    "ms_per_step": round(ep["dt"] / args.steps * 1e3, 4)}
            except Exception as e:  # an extra must not lose the headline
                extras["ep_weak_scaling"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    per = main_res["per"]
    t_gu, t_dn = per["gate_up"]["mean_ms"], per["down"]["mean_ms"]
    achieved = (f_gu + f_dn) / ((t_gu + t_dn) * 1e-3) / 1e12
    # roofline of the step's two launches (this rank's at N > 1): MFMA-bound unless the arithmetic
    # intensity puts the HBM roof (algorithmic bytes x 8 TB/s) below the MFMA peak
    if (f_gu + f_dn) / b_step * HBM_GBS / 1e3 < peak:
        gbs = b_step / ((t_gu + t_dn) * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_GBS, "unit": "GB/s", "frac": round(gbs / HBM_GBS, 4),
                "achieved_tflops": round(achieved, 2)}
    else:
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4)}
    value = main_res["total_flops"] * args.steps / main_res["dt"] / 1e12
    pmc = load_pmc_traffic(cfg) if world == 1 else None  # the committed PMC passes are single-GPU runs

    if rank == 0 and world == 1:
        for gg in ("gate_up", "down"):
            b = main_res["bytes"][gg]
            f = main_res["flops"][gg]
            extras[gg] = {"gflop": round(f / 1e9, 3), "median_ms": round(per[gg]["median_ms"], 4),
                          "tflops_median": round(f / (per[gg]["median_ms"] * 1e-3) / 1e12, 2),
                          "tiles": main_res["tiles"][gg], "algorithmic_MB": round(b / 1e6, 1),
                          "AI_flop_per_B": round(f / b, 1),
                          "roof_tflops": round(min(peak, f / b * HBM_GBS / 1e3), 1)}
    if world == 1 and args.extras:
        for x in [e for e in args.extras.split(",") if e and e != cfg]:
            r = run_config(x, 0, args.extras_warmup, False)
            pk = PEAK_TFLOPS[CONFIGS[x]["peak"]]
            tt = r["per"]["gate_up"]["median_ms"] + r["per"]["down"]["median_ms"]
            ff = r["flops"]["gate_up"] + r["flops"]["down"]
            bb = r["bytes"]["gate_up"] + r["bytes"]["down"]
            extras[x] = {"tflops": round(ff / (tt * 1e-3) / 1e12, 2),
                         "gate_up_tflops": round(r["flops"]["gate_up"] / (r["per"]["gate_up"]["median_ms"] * 1e-3) / 1e12, 2),
                         "down_tflops": round(r["flops"]["down"] / (r["per"]["down"]["median_ms"] * 1e-3) / 1e12, 2),
                         "ms_per_step": round(tt, 4), "variant": r["variant"]}
            if ff / bb * HBM_GBS / 1e3 < pk:  # the HBM roof binds (small batches: the weight stream)
                gbs = bb / (tt * 1e-3) / 1e9
                extras[x].update(bound="hbm", roofline_frac=round(gbs / HBM_GBS, 4), achieved_gbs=round(gbs, 1),
                                 algorithmic_MB=round(bb / 1e6, 1), peak_gbs=HBM_GBS)
            else:
                extras[x].update(bound="mfma", roofline_frac=round(ff / (tt * 1e-3) / 1e12 / pk, 4), peak_tflops=pk)

    if world == 1 and not args.no_moe_layer and CONFIGS[cfg].get("model", "qwen2_moe") == "qwen2_moe":
        try:  # the MoE layer around the path: not part of value
            from mxmoe_amd.moe import qwen2_layer_bench

            extras["moe_layer"] = {
                "what": "qwen2_moe layer-11 MoE FFN at bs 8192 (LP-1 mixed, random weights, routed histogram), planned "
                        "launches (moe.PlannedForward): quant_act -> gate_up -> SiLU-mul + quant -> down -> combine, "
                        "device us (median of alternating rounds); fused = the gate_up epilogue writes silu(g)*u "
                        "(MXMOE_GG_EPI_SILU_MUL) and only the quantisation follows",
                **qwen2_layer_bench(rounds=2, iters=20)}
            torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001 - an extra must not sink the headline line
            extras["moe_layer"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        try:  # the same layer at bs 512, where the gate_up call runs on the small-batch kernel (wo3)
            from mxmoe_amd.moe import qwen2_layer_bench

            extras["moe_layer_bs512"] = {
                "what": "as moe_layer at bs 512; interleaved = the fused layout through the plain epilogue + the "
                        "interleaved-input SiLU pass (the small-batch form before round 6, when wo3 had no SiLU "
                        "epilogue)",
                **qwen2_layer_bench(rounds=2, iters=20, bs=512, interleaved=True)}
            torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001
            extras["moe_layer_bs512"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        try:  # the reference's small-batch MoE scheme (w4a16 experts + 1/16 w8a8) at bs 512: the weight-only
            # gate_up problems take wo3's WO_SILU build when fused
            from mxmoe_amd.moe import qwen2_layer_bench

            extras["moe_layer_w4a16_w8a8_bs512"] = qwen2_layer_bench(rounds=2, iters=20, bs=512, interleaved=True,
                                                                     scheme="w4a16_w8a8")
            torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001
            extras["moe_layer_w4a16_w8a8_bs512"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        try:  # the same on the DeepSeek-V2-Lite mixed layer (64 routed experts, top-6, merged shared experts)
            from mxmoe_amd.moe import qwen2_layer_bench

            extras["moe_layer_ds2"] = qwen2_layer_bench(rounds=2, iters=20, model="ds2")
            torch.cuda.empty_cache()
        except Exception as e:  # noqa: BLE001
            extras["moe_layer_ds2"] = {"error": f"{type(e).__name__}: {e}"[:300]}

    if world == 1 and not args.no_scaling_sim:
        from mxmoe_amd.harness import build_layer_inputs as _bli, ep_scaling_sim, time_reference_abi

        asref = {}
        li = {gg: _bli(main_res["shapes"][gg], device=dev, seed=42 + (gg == "down")) for gg in ("gate_up", "down")}
        sim = ep_scaling_sim(li["gate_up"], li["down"], variant=args.variant if args.variant >= 0 else None,
                             shared=CONFIGS[cfg].get("model") != "mixtral")
        for gg in ("gate_up", "down"):
            asref[gg] = round(time_reference_abi(li[gg]), 4)
        del li
        torch.cuda.empty_cache()
        extras["strong_scaling_sim"] = {
            "what": "compute-only T1 / max-rank T_G of the N > 1 headline's plan (dist.ep_layer_plan: gate_up + down "
                    "per rank), each rank timed on this one GPU (ranks are independent GPUs); the all-gather of "
                    "the down outputs is not included (MB received per rank listed)",
            **sim}
        f = main_res["flops"]
        extras["as_reference"] = {
            "what": "groupgemm_mxmoe (reference FuncType) called back to back: per call the D2H pointer gather + one "
                    "sync, the plan (cached per device for repeated shapes; pointers re-validated) and the launch, wall ms",
            "gate_up_ms": asref["gate_up"], "down_ms": asref["down"],
            "tflops": round((f["gate_up"] + f["down"]) / ((asref["gate_up"] + asref["down"]) * 1e-3) / 1e12, 2)}

    if world == 1:
        ref = {"hardware": "RTX-4090", "source": "reference README media/final-perf.png read by eye (BASELINE.md §1)"}
        for c in [cfg] + [x for x in args.extras.split(",") if x in extras]:
            if c in REFERENCE_CHART_TFLOPS:
                mine = value if c == cfg else extras[c]["tflops"]
                ref[c] = {"reference_tflops": REFERENCE_CHART_TFLOPS[c], "ratio": round(mine / REFERENCE_CHART_TFLOPS[c], 2)}
        extras["reference_published_chart"] = ref

    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, main_res["shapes"])

    if rank == 0:
        out = {
            "metric": "GroupGEMM TFLOP/s + %roofline, qwen2_moe layer-11 bs=8192 at 1/8 GPU",
            "value": round(value, 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_s": args.settle_s,
            "materialise_after_plan": bool(args.materialise_after_plan),
            "ms_per_step": round(main_res["dt"] / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": CONFIGS[cfg]["dtype"],
            "data": "synthetic: uniform(-1,1) fp16 inputs (seeded) -> RTN per-row quantised + pack_wxax for "
                    "quantised problems; routed M_e = " + ("reference's committed bs=8192 histogram"
                                                         if not (cfg.startswith("ds2") or "model" in CONFIGS[cfg]) else
                                                         "seeded multinomial (SURVEY.md 8d)"),
            "config": {"workload": CONFIGS[cfg]["name"] + (f", one layer split by expert over {world} GPUs "
                                                          f"({'RCCL' if backend == 'nccl' else backend} all-gather "
                                                          f"of the layer outputs)" if world > 1 else ""),
                       "model": {"mixtral": "Mixtral-8x7B", "qwen2_moe_57b": "Qwen2-57B-A14B"}.get(
                           CONFIGS[cfg].get("model"),
                           "DeepSeek-V2-Lite" if cfg.startswith("ds2") else "qwen2_moe (Qwen1.5-MoE-A2.7B)")
                       + " MoE GroupGEMMs", "global_batch": CONFIGS[cfg].get("bs", 8192),
                       "seq_len": None, "parallelism": f"ep{world}+allgather" if world > 1 else "single",
                       "problems_per_call": len(main_res["shapes"]["gate_up"]), "variant": main_res["variant"],
                       "variant_name": nat.list_variants()[main_res["variant"]].split()[1]},
            "roofline": {**roof,
                         "traffic": pmc.get("hbm_bytes_per_step") if isinstance(pmc, dict) else None,
                         "traffic_source": pmc.get("_source") if isinstance(pmc, dict) else None,
                         "kernel": kernel_symbol(nat.list_variants()[main_res["variant"]].split()[1])
                         + " (gate_up + down launches; achieved = sum FLOPs / sum mean launch time)",
                         "launch_ms": {"gate_up": round(t_gu, 4), "down": round(t_dn, 4)}},
            "cpu_baseline": cpu,
            "extras": extras,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def kernel_symbol(variant_name: str) -> str:
    """Kernel template a variant launches (the name rocprofv3 reports)."""
    return {"v0": "mxmoe::gg_fused_kernel", "v2": "mxmoe::gg_v2_kernel", "v3": "mxmoe::gg_v3_kernel"}.get(
        variant_name[:2], variant_name)


if __name__ == "__main__":
    main()
