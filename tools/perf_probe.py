"""Quick perf probe: every compiled variant on the qwen2_moe layer-11 bs=8192 GroupGEMMs.

python tools/perf_probe.py [--cfg fp16,w8a8,w4a4,mixed] [--variants 0,1,2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.harness import bench_call, build_layer_inputs  # noqa: E402
from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="fp16,w8a8,w4a4,mixed")
    ap.add_argument("--variants", default=None)
    ap.add_argument("--iters", type=int, default=30)
    args = ap.parse_args()
    variants = list(range(nat.variant_count())) if args.variants is None else [int(x) for x in args.variants.split(",")]
    cfgs = {"fp16": dict(), "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
            "mixed": dict(qconfig=mixed_qconfig_lp1())}
    res = []
    for name in args.cfg.split(","):
        wl = load_workload(qwen2_layer11_workload(8192, **cfgs[name]))["layer-11"]
        for gg in ("gate_up", "down"):
            t0 = time.time()
            inp = build_layer_inputs(wl[gg])
            torch.cuda.synchronize()
            for v in variants:
                r = bench_call(inp, v, warmup=10, iters=args.iters)
                r.update(cfg=name, gg=gg, variant=v, gflop=inp.flops / 1e9)
                res.append(r)
                print(json.dumps(r), flush=True)
            del inp
            torch.cuda.empty_cache()
            print(f"# {name} {gg} setup+bench {time.time() - t0:.1f}s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "perf_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
