"""Tile timeline of one GroupGEMM launch (variant abl_v2s_trace, mxmoe_gg_debug_trace).

python tools/tile_trace.py --cfg fp16 --gg gate_up [--bs 8192] [--dump out.npy]

Prints where the launch's CU-time goes: mainloop, epilogue (stores drained), the gap between a
CU's consecutive blocks (block retire -> next block's first instruction: dispatch + setup), and
the idle time before a CU's first / after its last block. Timestamps are s_memrealtime (100 MHz).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import build_layer_inputs, time_launches  # noqa: E402
from mxmoe_amd.workload import QShape, load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402

TICK_US = 0.01


def fetch(nblocks: int, reset: bool) -> np.ndarray:
    buf = np.zeros((min(nblocks, 32768), 4), dtype=np.uint64)
    nat.check(nat.lib().mxmoe_gg_debug_trace(ctypes.c_void_p(buf.ctypes.data), buf.nbytes, int(reset)))
    return buf


def analyse(tr: np.ndarray) -> dict:
    ok = (tr[:, 0] != 0) & (tr[:, 2] != 0)  # padding blocks (prob < 0) leave only a start mark
    tr = tr[ok]
    t0 = int(tr[:, 0].min())
    st, ml, en = ((tr[:, i].astype(np.int64) - t0) for i in range(3))
    hw = tr[:, 3]
    xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
    hid = hw & np.uint64(0xFFFFFFFF)
    cu_key = (xcc << np.uint64(16)) | (((hid >> np.uint64(8)) & np.uint64(0xF)) << np.uint64(8)) | \
        (((hid >> np.uint64(12)) & np.uint64(0x1)) << np.uint64(4)) | ((hid >> np.uint64(13)) & np.uint64(0x7))
    span = int(en.max())
    info = hw >> np.uint64(36)
    qt, cls, nst = (info & np.uint64(0xF)).astype(int), ((info >> np.uint64(4)) & np.uint64(0xFF)).astype(int), \
        (info >> np.uint64(12)).astype(int)
    dur = (en - st) * TICK_US
    per_class = {}
    for key in sorted(set(zip(qt.tolist(), cls.tolist()))):
        mk = (qt == key[0]) & (cls == key[1])
        per_class[f"q{key[0]}c{key[1]}"] = {"n": int(mk.sum()), "us_per_stage": round(float(np.median(dur[mk] / np.maximum(nst[mk], 1))), 3),
                                            "median_us": round(float(np.median(dur[mk])), 2),
                                            "median_mark1_us": round(float(np.median((ml - st)[mk])) * TICK_US, 2)}
    xload = [round(float(dur[xcc == x].sum()) / 32, 1) for x in range(8)]
    per_cu = defaultdict(list)
    for i, k in enumerate(cu_key.tolist()):
        per_cu[k].append(i)
    gaps, head, tail = 0, 0, 0
    for idx in per_cu.values():
        idx.sort(key=lambda i: st[i])
        head += st[idx[0]]
        tail += span - en[idx[-1]]
        for a, b in zip(idx, idx[1:]):
            gaps += max(0, st[b] - en[a])
    ncu = len(per_cu)
    tot = ncu * span
    has_ml = ml >= st  # blocks without a mainloop mark (v5 / WO bodies) count as mainloop
    mloop = np.where(has_ml, ml - st, en - st).sum()
    epi = np.where(has_ml, en - ml, 0).sum()
    return {"blocks": int(ok.sum()), "cus": ncu, "span_us": round(span * TICK_US, 2),
            "mainloop_frac": round(mloop / tot, 4), "epilogue_frac": round(epi / tot, 4),
            "gap_frac": round(gaps / tot, 4), "head_frac": round(head / tot, 4), "tail_frac": round(tail / tot, 4),
            "blocks_per_cu": round(len(st) / ncu, 2),
            "median_mainloop_us": round(float(np.median(np.where(has_ml, ml - st, en - st))) * TICK_US, 2),
            "median_epilogue_us": round(float(np.median(np.where(has_ml, en - ml, 0))) * TICK_US, 2),
            "median_gap_us": round(gaps / max(1, len(st) - ncu) * TICK_US, 2),
            "xcd_load_us": xload, "per_class": per_class}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="fp16")
    ap.add_argument("--gg", default="gate_up")
    ap.add_argument("--bs", type=int, default=8192)
    ap.add_argument("--dense", default="")
    ap.add_argument("--dump", default="")
    ap.add_argument("--env", default="", help="KEY=VALUE set before planning (e.g. MXMOE_GG_XCD_BALANCE=0)")
    ap.add_argument("--variant-name", default="abl_v2s_trace", help="a V2_TRACE build of the lab library")
    args = ap.parse_args()
    if args.env:
        k, v = args.env.split("=", 1)
        os.environ[k] = v
    kw = {"fp16": {}, "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
          "mixed": dict(qconfig=mixed_qconfig_lp1()), "w4a16": dict(qstr="w4a16_g128_asym"),
          "w4a16c": dict(qstr="w4a16_g-1_sym"), "w4a16ga": dict(qstr="w4a16_g-1_asym"), "w4a16_w8a8": {}}[args.cfg]
    if args.cfg == "w4a16_w8a8":  # bench config w4a16_w8a8_bs512's scheme
        from mxmoe_amd.workload import w4a16_w8a8_qconfig

        kw = dict(qconfig=w4a16_w8a8_qconfig())
    if args.dense:
        bits = {"fp16": 16, "w8a8": 8, "w4a4": 4}[args.cfg]
        shapes = [QShape([int(x) for x in args.dense.split(",")], bits, bits)]
    else:
        shapes = load_workload(qwen2_layer11_workload(args.bs, **kw))["layer-11"][args.gg]
    inp = build_layer_inputs(shapes)
    trace_v = [ln.split()[1] for ln in nat.list_variants()].index(args.variant_name)
    gg = GroupGemm(inp.problems, variant=trace_v)
    t = time_launches(gg.launch, warmup=20, iters=50)
    fetch(0, reset=True)
    gg.launch()
    torch.cuda.synchronize()
    tr = fetch(max(gg.info.grid, gg.info.tile_slots), reset=False)
    res = {"variant": args.variant_name, "cfg": args.cfg, "gg": args.dense or args.gg, "bs": args.bs, "env": args.env, "event_median_ms": round(t["median_ms"], 4)}
    res.update(analyse(tr))
    print(json.dumps(res), flush=True)
    if args.dump:
        np.save(args.dump, tr)


if __name__ == "__main__":
    main()
