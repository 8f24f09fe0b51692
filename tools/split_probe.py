"""Probe: a mixed w4a4 + w8a8 call as ONE fused launch (the reference's design: per-tile qtype branch,
compose_kernel.py:150-295) against the same problems split by quant type into two launches, each on
the AUTO variant of its own subset (w8a8 -> v2s / v2s3, w4a4-only -> v3 2-WG/CU), either back to back
on one stream or concurrently on two streams joined by events.

python tools/split_probe.py [--cfg mixed|ds2_mixed] [--rounds 10] [--iters 20] > gpurun_out/split_probe.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import build_layer_inputs, time_launches  # noqa: E402
from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="mixed", choices=["mixed", "ds2_mixed", "w4a16_w8a8"])
    ap.add_argument("--bs", type=int, default=8192)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--split", default="qtype", choices=["qtype", "shared"],
                    help="shared: the largest-M problem (the shared expert) on v2x (variant 1) vs the rest on AUTO")
    args = ap.parse_args()
    for gg_name in ("gate_up", "down"):
        if args.cfg == "ds2_mixed":
            from mxmoe_amd.workload import ds2_mixed_qconfig, ds2_workload

            shapes = load_workload(ds2_workload(args.bs, qconfig=ds2_mixed_qconfig()))["layer-1"][gg_name]
        elif args.cfg == "w4a16_w8a8":  # split: weight-only problems (-> wo3 at small batch) vs w8a8
            from mxmoe_amd.workload import w4a16_w8a8_qconfig

            shapes = load_workload(qwen2_layer11_workload(args.bs, qconfig=w4a16_w8a8_qconfig()))["layer-11"][gg_name]
        else:
            shapes = load_workload(qwen2_layer11_workload(args.bs, qconfig=mixed_qconfig_lp1()))["layer-11"][gg_name]
        inp = build_layer_inputs(shapes)
        probs = inp.problems
        if args.split == "shared":
            big = max(range(len(shapes)), key=lambda i: shapes[i].M)
            p8 = [probs[big]]
            p4 = [p for i, p in enumerate(probs) if i != big]
            g8, g4 = GroupGemm(p8, variant=1), GroupGemm(p4)
        else:
            p8 = [p for p, s in zip(probs, shapes) if s.a_bits == 8]
            p4 = [p for p, s in zip(probs, shapes) if s.a_bits == (16 if args.cfg == "w4a16_w8a8" else 4)]
            g8, g4 = GroupGemm(p8), GroupGemm(p4)
        fused = GroupGemm(probs)
        main_s = torch.cuda.current_stream()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

        def seq():
            g8.launch()
            g4.launch()

        def conc():
            ev0 = torch.cuda.Event()
            ev0.record(main_s)
            s1.wait_event(ev0)
            s2.wait_event(ev0)
            g8.launch(s1)
            g4.launch(s2)
            e1, e2 = torch.cuda.Event(), torch.cuda.Event()
            e1.record(s1)
            e2.record(s2)
            main_s.wait_event(e1)
            main_s.wait_event(e2)

        arms = {"fused": fused.launch, "split_seq": seq, "split_2streams": conc}
        for fn in arms.values():  # settle clocks
            time_launches(fn, warmup=5, iters=20)
        samples = {k: [] for k in arms}
        per = max(1, args.iters // args.rounds)
        for _ in range(args.rounds):
            for k, fn in arms.items():
                samples[k].append(time_launches(fn, warmup=1, iters=per)["median_ms"])
        t8 = time_launches(g8.launch, warmup=5, iters=20)["median_ms"]
        t4 = time_launches(g4.launch, warmup=5, iters=20)["median_ms"]
        res = {"cfg": args.cfg, "gg": gg_name, "variants": {"fused": fused.variant, "w8a8": g8.variant, "w4a4": g4.variant},
               "w8a8_alone_ms": round(t8, 4), "w4a4_alone_ms": round(t4, 4)}
        for k, ts in samples.items():
            med = statistics.median(ts)
            res[k] = {"median_ms": round(med, 4), "spread_ms": round(max(ts) - min(ts), 4),
                      "tops": round(inp.flops / (med * 1e-3) / 1e12, 1)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
