"""Does the MI355X performance table's cost model (the reference's get_runtime_cost restated,
bits_solver.py:518-542: inc x num_tiles per problem) predict a measured GroupGEMM call? The
committed table (measured on calls of identical 4 x 4-tile problems) against qwen2_moe layer-11
calls at bs=8192: the prediction must land within 25 % of the measured time and rank
the quantisation strategies of a call like the measurement does (what the ILP needs from it)."""
from __future__ import annotations

import json
from pathlib import Path

import pytest
import torch

from mxmoe_amd import perf_table as pt
from mxmoe_amd.groupgemm import GroupGemm
from mxmoe_amd.harness import build_layer_inputs, time_launches
from mxmoe_amd.workload import load_workload, qwen2_layer11_workload

pytestmark = pytest.mark.gpu
TABLE = Path(pt.__file__).resolve().parent / "workloads" / "performance_table_mi355x.json"


def predicted_ms(shapes, table, tiles):
    live = [s for s in shapes if s.M > 0]
    q = live[0].qcfg
    first = next(iter(table[q]["2"].values()))["first_iter_cost"]
    return first + sum(pt.runtime_cost([[s]], [s.qcfg], table, tiles)[0][0][0] for s in live)


def test_cost_model_predicts_layer_calls():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    table = json.loads(TABLE.read_text())
    tiles = pt.tiles_from_table(table)
    res = {}
    for bs in (8192, 4096):
        for cfg, kw in (("fp16", {}), ("w8a8", dict(qstr="w8a8_g-1_sym")), ("w4a4", dict(qstr="w4a4_g-1_sym"))):
            layer = load_workload(qwen2_layer11_workload(bs, **kw))["layer-11"]
            for gg in ("gate_up", "down"):
                inp = build_layer_inputs(layer[gg])
                meas = time_launches(GroupGemm(inp.problems).launch, warmup=10, iters=20)["median_ms"]
                res[(bs, cfg, gg)] = (predicted_ms(layer[gg], table, tiles), meas)
                del inp
                torch.cuda.empty_cache()
    print(json.dumps({f"{b}/{c}/{g}": {"predicted_ms": round(p, 4), "measured_ms": round(m, 4), "ratio": round(p / m, 3)}
                      for (b, c, g), (p, m) in res.items()}))
    for (b, c, g), (p, m) in res.items():
        assert 0.75 < p / m < 1.25, f"{b}/{c}/{g}: predicted {p:.4f} ms, measured {m:.4f} ms"
    # no strategy priced systematically high or low: the mean of predicted / measured - 1 over its four
    # calls (bs 8192 and 4096, gate_up and down). Round 6 re-measured the w4a4 / w8a8 / fp16 rows on
    # the AUTO kernels of the day (profiles/r06/perf/): w4a4 +9.0 %, w8a8 +2.4 %, fp16 +1.8 % (the
    # round-4 w4a4 row: +15.8 %); the bound leaves room for box-to-box spread
    for c in ("fp16", "w8a8", "w4a4"):
        bias = sum(p / m - 1 for (b, cc, g), (p, m) in res.items() if cc == c) / 4
        assert abs(bias) <= 0.12, (c, round(bias, 3))
    for g in ("gate_up", "down"):  # the ranking the ILP relies on: fp16 slowest, then the 8- / 4-bit pair
        pred = {c: res[(8192, c, g)][0] for c in ("fp16", "w8a8", "w4a4")}
        meas = {c: res[(8192, c, g)][1] for c in ("fp16", "w8a8", "w4a4")}
        assert max(pred, key=pred.get) == max(meas, key=meas.get) == "fp16", (g, pred, meas)
        # w8a8 (v2x) and w4a4 (v3) run within a few % of each other since round 3: a measured gap
        # under 5 % is a tie, which the model must then also predict as close (< 15 %); a wider
        # measured gap must be ranked the same way (round 5 had widened this band to 10 % / 20 %
        # instead of re-measuring the stale w4a4 row; round 6 re-measured it and restored the band)
        if abs(meas["w8a8"] / meas["w4a4"] - 1) <= 0.05:
            assert abs(pred["w8a8"] / pred["w4a4"] - 1) < 0.15, (g, pred, meas)
        else:
            assert (pred["w8a8"] < pred["w4a4"]) == (meas["w8a8"] < meas["w4a4"]), (g, pred, meas)
