"""Per-rank strong-scaling work lists timed with several variants (tile-fill study).

python tools/nslice_probe.py --cfg fp16 --variants 8,7
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mxmoe_amd.harness import build_layer_inputs, strong_scaling_sim  # noqa: E402
from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="fp16")
    ap.add_argument("--variants", default="8,7")
    args = ap.parse_args()
    kw = {"fp16": {}, "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
          "mixed": dict(qconfig=mixed_qconfig_lp1())}[args.cfg]
    layer = load_workload(qwen2_layer11_workload(8192, **kw))["layer-11"]
    for gg in ("gate_up", "down"):
        inp = build_layer_inputs(layer[gg])
        for v in [int(x) for x in args.variants.split(",")]:
            r = strong_scaling_sim(inp, variant=v)
            print(json.dumps({"cfg": args.cfg, "gg": gg, "variant": v, "t1_ms": r["t1_ms"],
                              **{G: r[G]["t_ms_max_rank"] for G in ("2", "4", "8")}}), flush=True)


if __name__ == "__main__":
    main()
