"""Time the MoE-layer plumbing kernels (include/mxmoe_moe.h) on qwen2_moe layer 11 at bs=8192.

python tools/moe_bench.py [--iters 50] > gpurun_out/moe_bench.jsonl

Routing: topk = 4 choices per token whose per-expert counts are the committed bs=8192 histogram
(the routed M_e of the GroupGEMM workload), shuffled over the tokens; activation quantisation per
expert from the LP-1 mixed qconfig (w4a4 -> int4, w8a8 -> int8; shared expert last). One JSON line
per kernel: device time (HIP events on the launch stream, median), algorithmic bytes (each byte a
kernel must read or write once), GB/s and the fraction of the 8 TB/s HBM roof.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd import moe  # noqa: E402
from mxmoe_amd.harness import time_launches  # noqa: E402
from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402

HBM_GBS = 8000.0
T, TOPK, E, H, N, NS = 8192, 4, 60, 2048, 1408, 5632


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = "cuda"
    layer = load_workload(qwen2_layer11_workload(T, qconfig=mixed_qconfig_lp1()))["layer-11"]
    counts = [s.M for s in layer["gate_up"][:E]]
    counts[0] += T * TOPK - sum(counts)  # the histogram's int() truncation: 6 slots short of T*topk
    g = torch.Generator().manual_seed(0)
    ids = torch.repeat_interleave(torch.arange(E, dtype=torch.int32), torch.tensor(counts))
    ids = ids[torch.randperm(ids.numel(), generator=g)].view(T, TOPK).contiguous().to(dev)
    tags1 = [moe.qtag_of(s.a_bits, s.gsize) for s in layer["gate_up"]]
    tags2 = [moe.qtag_of(s.a_bits, s.gsize) for s in layer["down"]]
    hidden = ((torch.rand(T, H, generator=g) * 2 - 1)).half().to(dev)
    routed = ((torch.rand(T * TOPK, 2 * N, generator=g) * 2 - 1) * 4).half().to(dev)
    shared = ((torch.rand(T, 2 * NS, generator=g) * 2 - 1) * 4).half().to(dev)
    y = ((torch.rand(T * TOPK, H, generator=g) * 2 - 1)).half().to(dev)
    ys = ((torch.rand(T, H, generator=g) * 2 - 1)).half().to(dev)
    w = torch.softmax(torch.rand(T, TOPK, generator=g), dim=1).to(dev)

    r = moe.route(ids, E)
    bufs = moe.route_device(ids, E)
    a1 = moe.quant_act(hidden, r, tags1, with_shared=True)
    a2 = moe.silu_mul_quant(routed, shared, r, tags2)
    slots = T * TOPK

    def bits(tag):
        return {moe.ACT_FP16: 16, moe.ACT_INT8: 8, moe.ACT_INT4: 4, moe.ACT_INT4_G128: 4}[tag]

    def out_bytes(rows, width, tag):
        sc = 0 if tag == moe.ACT_FP16 else 2 * rows * (width // 128 if tag == moe.ACT_INT4_G128 else 1)
        return rows * width * bits(tag) // 8 + sc

    rows = list(r.counts) + [T]
    q_bytes = (slots + T) * H * 2 + sum(out_bytes(m, H, t) for m, t in zip(rows, tags1))
    s_bytes = (slots * 2 * N + T * 2 * NS) * 2 + sum(
        out_bytes(m, wd, t) for m, wd, t in zip(rows, [N] * E + [NS], tags2))
    c_bytes = (slots + T) * H * 2 + slots * (4 + 4) + T * H * 2
    r_bytes = slots * 4 * 4 + E * 4
    cases = [
        ("route", lambda: moe.route_device(ids, E, out=bufs), r_bytes, "device kernel only"),
        ("quant_act", a1.relaunch, q_bytes, "LP-1 gate_up activation qcfg, 61 segments"),
        ("silu_mul_quant", a2.relaunch, s_bytes, "LP-1 down activation qcfg, routed + shared launches"),
        ("combine", lambda: moe.combine(y, r, w, ys), c_bytes, "top-4 weighted sum + shared expert"),
    ]
    for name, fn, nbytes, note in cases:
        t = time_launches(fn, warmup=10, iters=args.iters)
        us = t["median_ms"] * 1e3
        gbs = nbytes / (us * 1e-6) / 1e9
        print(json.dumps({"kernel": name, "median_us": round(us, 2), "MB": round(nbytes / 1e6, 2),
                          "GB_s": round(gbs, 1), "hbm_frac": round(gbs / HBM_GBS, 4), "note": note}), flush=True)


if __name__ == "__main__":
    main()
