"""The planner's own tile-time model applied to a plan's tile table (mxmoe_gg_plan_tiles): per XCD
the queue (blocks 8 i + x) taken by `chunk` workgroup slots in order, the modelled makespan against
the mean per-slot load (1.0 = perfectly level), and where each problem's tiles landed (the XCDs an
expert spans: its A / B panels are re-read from each of those L2s).

python tools/plan_model.py --cfg fp16 --gg down [--bs 8192] [--env MXMOE_GG_XCD_PACK=1]
(env knobs are read by the lab library only: MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so)
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stage_time(s, cls: int, geom=(256, 256, 128), tail=(128, 64)) -> float:
    """gg_api.hip plan_host::stage_time for the fp16 / int8 / int4 bodies of the v2 kernels."""
    rows = geom[0] if cls == 0 else tail[cls - 1]
    cols, bkb = geom[1], geom[2]
    fp = s.a_bits == 16
    kel = bkb * 8.0 / (16 if fp else 8 if s.w_bits == 8 else 4)
    rate = 128 if fp else 256
    return max((rows + cols) * bkb, 2.0 * rows * cols * kel / rate) + 24576.0


def model(shapes, tiles, rows, chunk: int = 32) -> dict:
    import numpy as np

    P = len(shapes)
    xcd_t = [[] for _ in range(8)]
    spans = [set() for _ in range(P)]
    for b, t in enumerate(tiles):
        if t[0] < 0:
            continue
        i = int(rows[t[0]])  # table row -> the caller's problem index
        dt = stage_time(shapes[i], int(t[3]) & 0xFF) * (int(t[5]) - int(t[4]))
        xcd_t[b % 8].append(dt)
        spans[i].add(b % 8)
    fin, load = [], []
    for q in xcd_t:
        slot = [0.0] * chunk
        f = 0.0
        for dt in q:
            s0 = heapq.heappop(slot)
            heapq.heappush(slot, s0 + dt)
            f = max(f, s0 + dt)
        fin.append(f)
        load.append(sum(q))
    mean = sum(load) / (8 * chunk)
    return {"makespan_over_mean": round(max(fin) / mean, 4), "xcd_finish_over_mean": [round(f / mean, 3) for f in fin],
            "xcd_load_over_mean": [round(l / chunk / mean, 3) for l in load],
            "routed_xcd_span_mean": round(float(np.mean([len(s) for s in spans[:-1] if s])), 2),
            "shared_xcd_span": len(spans[-1])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="fp16")
    ap.add_argument("--gg", default="down")
    ap.add_argument("--bs", type=int, default=8192)
    ap.add_argument("--env", default="", help="K=V[,K=V]: planner knobs (lab library)")
    ap.add_argument("--variant", default="auto")
    args = ap.parse_args()
    for kv in filter(None, args.env.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    from mxmoe_amd import _native as nat
    from mxmoe_amd.workload import load_workload, mixed_qconfig_lp1, qwen2_layer11_workload

    kw = {"fp16": {}, "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
          "mixed": dict(qconfig=mixed_qconfig_lp1())}
    if args.cfg == "ds2_mixed":
        from mxmoe_amd.workload import ds2_mixed_qconfig, ds2_workload

        shapes = load_workload(ds2_workload(args.bs, qconfig=ds2_mixed_qconfig()))["layer-1"][args.gg]
    else:
        shapes = load_workload(qwen2_layer11_workload(args.bs, **kw[args.cfg]))["layer-11"][args.gg]
    probs = [nat.GGProblemC(A=0, B=0, scale_a=0, scale_b=0, C=0, M=s.M, N=s.N, K=s.K, a_bits=s.a_bits,
                            w_bits=s.w_bits, gsize=s.gsize, sym=int(s.sym), fmt=0, lda=0, ldb=0, ldc=0) for s in shapes]
    arr = (nat.GGProblemC * len(probs))(*probs)
    v = nat.resolve_variant(arr, len(probs), -1 if args.variant == "auto" else int(args.variant))
    tiles, rows = nat.plan_tiles(probs, v)
    out = {"cfg": args.cfg, "gg": args.gg, "bs": args.bs, "env": args.env, "variant": nat.list_variants()[v].split()[1]}
    out.update(model(shapes, tiles, rows))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
