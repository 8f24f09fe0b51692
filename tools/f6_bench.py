"""w4a4 layer calls on the int4 path (AUTO: v3) against the fp6-image path (gg_f6.h): GEMM alone
(A images resident) and A re-encoding + GEMM, per call, same process, alternating order.

python tools/f6_bench.py [--cfg w4a4|ds2_w4a4] [--bs 8192] [--reps 3] [--out gpurun_out/f6/bench.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import F6Layer, build_layer_inputs, time_launches  # noqa: E402
from mxmoe_amd.workload import ds2_workload, load_workload, qwen2_layer11_workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="w4a4")
    ap.add_argument("--bs", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--f6-variants", default="", help="comma-separated variant names to time as extra fp6 arms")
    args = ap.parse_args()
    if args.cfg == "ds2_w4a4":
        wl = load_workload(ds2_workload(args.bs, qstr="w4a4_g-1_sym"))["layer-1"]
    else:
        wl = load_workload(qwen2_layer11_workload(args.bs, qstr="w4a4_g-1_sym"))["layer-11"]
    res = {"cfg": args.cfg, "bs": args.bs}
    for gg in ("gate_up", "down"):
        inp = build_layer_inputs(wl[gg])
        f6 = F6Layer(inp)
        g4 = GroupGemm(inp.problems)
        g6 = GroupGemm(f6.problems)
        arms = {"int4_auto": g4.launch, "f6_gemm": g6.launch, "f6_pack_gemm": lambda: (f6.pack_a(), g6.launch()),
                "f6_pack_only": f6.pack_a}
        names = [ln.split()[1] for ln in nat.list_variants()]
        for vn in filter(None, args.f6_variants.split(",")):
            arms[vn] = GroupGemm(f6.problems, variant=names.index(vn)).launch
        t = {k: [] for k in arms}
        for _ in range(args.reps):
            for k, fn in arms.items():
                t[k].append(time_launches(fn, 10, 30)["median_ms"])
        med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
        tflops = {k: inp.flops / (med[k] * 1e-3) / 1e12 for k in med if k != "f6_pack_only"}
        res[gg] = {"ms": {k: round(v, 4) for k, v in med.items()}, "tops": {k: round(v, 1) for k, v in tflops.items()},
                   "variants": {"int4_auto": g4.variant, "f6": g6.variant}, "reps_ms": t}
        print(gg, json.dumps(res[gg]["ms"]), json.dumps(res[gg]["tops"]), flush=True)
        del inp, f6, g4, g6
        torch.cuda.empty_cache()
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
