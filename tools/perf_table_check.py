"""The performance table's cost model (mxmoe_amd/perf_table.py, bits_solver.py:518-542 restated)
against measured qwen2_moe layer-11 GroupGEMM calls: predicted / measured per strategy and call,
as tests/test_perf_table_gpu.py checks it (one JSON line).

python tools/perf_table_check.py [--table mxmoe_amd/workloads/performance_table_mi355x.json] [--bs 8192]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from mxmoe_amd import perf_table as pt
    from mxmoe_amd.groupgemm import GroupGemm
    from mxmoe_amd.harness import build_layer_inputs, time_launches
    from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default=os.path.join(ROOT, "mxmoe_amd", "workloads", "performance_table_mi355x.json"))
    ap.add_argument("--bs", default="8192")
    args = ap.parse_args()
    table = json.load(open(args.table))
    tiles = pt.tiles_from_table(table)
    out = {"table": os.path.relpath(args.table, ROOT)}
    for bs in (int(b) for b in args.bs.split(",")):
        for cfg, kw in (("fp16", {}), ("w8a8", dict(qstr="w8a8_g-1_sym")), ("w4a4", dict(qstr="w4a4_g-1_sym"))):
            layer = load_workload(qwen2_layer11_workload(bs, **kw))["layer-11"]
            for gg in ("gate_up", "down"):
                inp = build_layer_inputs(layer[gg])
                g = GroupGemm(inp.problems)
                meas = time_launches(g.launch, warmup=10, iters=30)["median_ms"]
                live = [s for s in layer[gg] if s.M > 0]
                q = live[0].qcfg
                first = next(iter(table[q]["2"].values()))["first_iter_cost"]
                pred = first + sum(pt.runtime_cost([[s]], [s.qcfg], table, tiles)[0][0][0] for s in live)
                out[f"{bs}/{cfg}/{gg}"] = {"predicted_ms": round(pred, 4), "measured_ms": round(meas, 4),
                                           "ratio": round(pred / meas, 3), "variant": g.variant}
                del inp, g
                torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
