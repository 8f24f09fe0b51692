"""Launch one GroupGEMM call repeatedly (for rocprofv3 counter runs / A-B of variants).

python tools/kbench.py --cfg w8a8 --gg gate_up --variants 0,3 --iters 20 [--only shared|routed|all]
(--variants auto = the library's AUTO choice; 8@MXMOE_GG_XCD_BALANCE=0 = variant 8 planned with that env)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import build_layer_inputs, time_launches  # noqa: E402
from mxmoe_amd.workload import QShape, load_workload, mixed_qconfig_lp1, qwen2_layer11_workload  # noqa: E402


def padded(inp, pad):
    """The same inputs with every A / B row `pad` bytes longer (lda / ldb; fp16 and packed-int
    problems only): moves consecutive rows off a power-of-two stride."""
    import dataclasses

    from mxmoe_amd.harness import LayerInputs

    probs = []
    for p in inp.problems:
        if p.q.is_weight_only:
            probs.append(p)
            continue
        def pad_rows(t):
            u = t.view(torch.uint8)
            out = torch.zeros(u.shape[0], u.shape[1] + pad, dtype=torch.uint8, device=u.device)
            out[:, :u.shape[1]] = u
            return out.view(t.dtype), (u.shape[1] + pad) // 2
        A, lda = pad_rows(p.A)
        B, ldb = pad_rows(p.B)
        probs.append(dataclasses.replace(p, A=A, B=B, lda=lda, ldb=ldb))
    return LayerInputs(problems=probs, shapes=inp.shapes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="w8a8")
    ap.add_argument("--gg", default="gate_up")
    ap.add_argument("--variants", default="0,3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="all", choices=["all", "shared", "routed"])
    ap.add_argument("--rounds", type=int, default=5, help="round-robin rounds over the variants")
    ap.add_argument("--bs", type=int, default=8192, help="tokens (routed M_e scale with it)")
    ap.add_argument("--settle-s", type=float, default=1.0, help="seconds of load before timing")
    ap.add_argument("--pads", default="0", help="comma list of extra bytes per A / B row (row stride padding); "
                    "each pad gets its own input set, every variant runs on every set")
    ap.add_argument("--dense", default="", help="M,N,K: one dense problem (fp16 / w8a8 / w4a4) instead of the layer")
    args = ap.parse_args()
    kw = {"fp16": {}, "w8a8": dict(qstr="w8a8_g-1_sym"), "w4a4": dict(qstr="w4a4_g-1_sym"),
          "mixed": dict(qconfig=mixed_qconfig_lp1()), "w4a16": dict(qstr="w4a16_g128_asym"),
          "w4a16c": dict(qstr="w4a16_g-1_sym"), "w8a16": dict(qstr="w8a16_g-1_asym"),
          "w4a16ga": dict(qstr="w4a16_g-1_asym"), "w4a16gs": dict(qstr="w4a16_g128_sym"),
          "w4a4g128": dict(qstr="w4a4_g128_sym"), "w2a16": dict(qstr="w2a16_g128_asym"),
          "e4m3": dict(qstr="w8a8_g-1_sym_E4M3"), "bf16": dict(qstr="bf16"), "ds2_mixed": {},
          "w4a16_w8a8": {}}[args.cfg]
    if args.cfg == "w4a16_w8a8":  # bench config w4a16_w8a8_bs512's scheme (w4a16 + 1/16 w8a8)
        from mxmoe_amd.workload import w4a16_w8a8_qconfig

        kw = dict(qconfig=w4a16_w8a8_qconfig())
    if args.dense:
        bits = {"fp16": 16, "w8a8": 8, "w4a4": 4, "e4m3": 8, "bf16": 16}[args.cfg]
        fmt = {"e4m3": "E4M3", "bf16": "bf16"}.get(args.cfg, "")
        shapes = [QShape([int(x) for x in args.dense.split(",")], bits, bits, fmt=fmt)]
        args.gg = "dense_" + args.dense.replace(",", "x")
    elif args.cfg == "ds2_mixed":
        from mxmoe_amd.workload import ds2_mixed_qconfig, ds2_workload

        shapes = load_workload(ds2_workload(args.bs, qconfig=ds2_mixed_qconfig()))["layer-1"][args.gg]
    else:
        shapes = load_workload(qwen2_layer11_workload(args.bs, **kw))["layer-11"][args.gg]
    if args.only == "shared":
        shapes = shapes[-1:]
    elif args.only == "routed":
        shapes = shapes[:-1]
    base = build_layer_inputs(shapes)
    inputs = [(pad, base if pad == 0 else padded(base, pad)) for pad in (int(x) for x in args.pads.split(","))]
    inp = base
    ggs, labels = [], []
    for pad, spec in ((pad, spec) for pad, _ in inputs for spec in args.variants.split(",")):
        inp_p = dict(inputs)[pad]
        x, _, env = spec.partition("@")
        saved = {}
        if env:
            k, val = env.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = val
        ggs.append(GroupGemm(inp_p.problems, variant=None if x == "auto" else int(x)))  # None: AUTO
        labels.append(spec if pad == 0 else f"{spec}+pad{pad}")
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k)
            else:
                os.environ[k] = old
    # A/B without order bias: ~1 s of sustained load first (clocks settle), then round-robin rounds
    # over the variants; per-variant median over every round's samples
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.settle_s:
        for gg in ggs:
            gg.launch()
        torch.cuda.synchronize()
    samples = [[] for _ in ggs]
    per_round = max(1, args.iters // args.rounds)
    for _ in range(args.rounds):
        for k, gg in enumerate(ggs):
            t = time_launches(gg.launch, warmup=1, iters=per_round)
            samples[k].append(t["median_ms"])
    for gg, ts, lab in zip(ggs, samples, labels):
        med = statistics.median(ts)
        print(json.dumps({"variant": gg.variant, "spec": lab, "cfg": args.cfg, "gg": args.gg, "bs": args.bs, "only": args.only,
                          "median_ms": round(med, 4), "spread_ms": round(max(ts) - min(ts), 4),
                          "tiles": gg.total_tiles, "grid": gg.info.grid,
                          "tflops": round(inp.flops / (med * 1e-3) / 1e12, 1),
                          "gbs": round(inp.bytes_algorithmic() / (med * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
