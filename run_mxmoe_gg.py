"""run_mxmoe_gg.py — drop-in for the reference CLI (SeaCatComplexes/MxMoE run_mxmoe_gg.py:1-141).

Same flags (--model --dataset --qconfig --tile_config --qstr --bs --layer), same qcfg-list and
workload-path rules, same CSV schema. What changes is the middle: the reference generates CUDA
sources (TemplateGenerator), runs cmake/ninja and execs ./build/test; here the MI355X kernels are a
compiled variant table in mxmoe_amd/lib/libmxmoe_gg.so, the tile_config picks the nearest variant,
and the bench runs in-process on the GPU.

  step 1  workload JSON   -> out/workloads/{model}-{dataset}-{bs}{suffix}        (gen_workload.py)
  step 2  variant select  -> tile_config JSON (either exporter or per-qcfg form) or every variant
  step 3  bench / check   -> out/bench/{model}-{dataset}-{bs}{suffix}-layer-L-{gate_up|down}.csv
                             kernel_name,avg_time,TFLOPS,speedup (test.cu:855-865); speedup is vs
                             the vendor-library baseline (per-problem torch.matmul fp16 = hipBLASLt /
                             rocBLAS), the role cutlass GemmGrouped plays in the reference (test.cu:774-781)

Gate traces: --trace PATH, else calib/gate/{model}/{dataset}/4096/moe-gate.json (gen_workload.py:23-31)
if present, else the committed qwen2_moe bs=8192 histogram for qwen2_moe / a seeded
synthetic trace (workload.synthetic_trace) for ds2, qwen2_moe_57b and mixtral.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mxmoe_amd.qconfig import get_qcfg_list, load_qconfig  # noqa: E402
from mxmoe_amd.workload import (MODEL_ID_TO_LAYERS, generate_workload_from_trace, load_workload,  # noqa: E402
                                qwen2_hist, qwen2_layer11_trace, save_workload, synthetic_trace)

CUR_DIR = ROOT


def find_trace(model: str, dataset: str, layer: int, explicit: str | None) -> dict:
    if explicit:
        with open(explicit) as f:
            return json.load(f)
    p = os.path.join(CUR_DIR, "calib", "gate", model, dataset, "4096", "moe-gate.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    if model == "qwen2_moe":
        t = qwen2_layer11_trace()
        h = t.pop("layer-11")
        for li in range(MODEL_ID_TO_LAYERS[model]):  # the only routing data in the reference (§8d)
            t[f"layer-{li}"] = h
        return t
    if model in ("ds2", "qwen2_moe_57b", "mixtral"):
        t = synthetic_trace(model)
        h = t.pop("layer-1")
        for li in range(MODEL_ID_TO_LAYERS[model]):
            t[f"layer-{li}"] = h
        return t
    raise FileNotFoundError(f"no gate trace for {model}/{dataset}: pass --trace")


def workload_suffix(args) -> tuple[str, dict, list]:
    if args.qconfig is not None:
        qcfg_list = sorted(get_qcfg_list(args.qconfig, args.layer))
        suffix = "-" + args.qconfig.split("wbits")[1].split(".json")[0] + ".json" if "wbits" in args.qconfig else ".json"
        return suffix, dict(qconfig=load_qconfig(args.qconfig)), qcfg_list
    if args.qstr is not None:
        return f"-{args.qstr}.json", dict(qstr=args.qstr), [args.qstr]
    return "-fp16.json", {}, ["fp16"]


def main(argv=None):
    ap = argparse.ArgumentParser(description="Bench workloads for the MI355X groupgemm kernels.")
    ap.add_argument("--model", type=str, default="qwen2_moe", help="Model ID.")
    ap.add_argument("--dataset", type=str, default="wiki2", help="Dataset ID.")
    ap.add_argument("--qconfig", type=str, default=None, help="Path to the quantization config file.")
    ap.add_argument("--tile_config", type=str, default=None, help="Path to the tile config file.")
    ap.add_argument("--qstr", type=str, default=None, help="Short string to represent quantization config.")
    ap.add_argument("--bs", type=int, default=512, help="Batch size.")
    ap.add_argument("--layer", type=int, default=-1, help="Layer index.")
    ap.add_argument("--trace", type=str, default=None, help="Gate trace JSON (default: see module doc).")
    ap.add_argument("--mode", choices=["bench", "check"], default="bench")
    ap.add_argument("--variants", type=str, default=None, help="comma list (default: tile_config or all)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-baseline", action="store_true")
    ap.add_argument("--cpu-plumbing", action="store_true",
                    help="no GPU: write the workload JSON and time the per-problem torch.matmul fp16 baseline on "
                         "the host (BASELINE configs[0]: bs=128 plumbing); the HIP kernels are not run")
    args = ap.parse_args(argv)

    suffix, wl_kw, qcfg_list = workload_suffix(args)
    workload_path = f"{CUR_DIR}/out/workloads/{args.model}-{args.dataset}-{args.bs}{suffix}"
    layers = list(range(MODEL_ID_TO_LAYERS[args.model])) if args.layer == -1 else [args.layer]
    trace = find_trace(args.model, args.dataset, args.layer, args.trace)
    print(f"qcfg_list: {qcfg_list}")

    import torch

    from mxmoe_amd import _native as nat
    from mxmoe_amd.harness import build_layer_inputs, time_launches, write_csv
    from mxmoe_amd.check import check_sampled
    from mxmoe_amd.groupgemm import GroupGemm
    from mxmoe_amd.tile_config import parse_tile_config_json, select_variant

    if args.cpu_plumbing:
        return cpu_plumbing(args, trace, layers, wl_kw, workload_path, suffix)
    nat.lib()  # fails loudly if the HIP library is missing
    result = {"qcfg_list": qcfg_list, "variants": {}, "csv": []}
    for layer in layers:
        print(f"Processing Layer {layer}...")
        wl = generate_workload_from_trace(trace, args.bs, layer, **wl_kw)
        if args.model == "qwen2_moe" and args.bs == 8192 and not args.trace:
            h = qwen2_hist()["M"]  # pin the committed M_e (int(p*T*topk) truncation differs by <= 1 row)
            for gg in ("gate_up", "down"):
                for p, m in zip(wl[f"layer-{layer}"][gg][:-1], h):
                    p["shape"][0] = m
        save_workload(wl, workload_path)
        print(f"Save generated workloads to `{workload_path}`")
        if args.variants:
            variants = [int(v) for v in args.variants.split(",")]
        elif args.tile_config:
            tiles = parse_tile_config_json(args.tile_config, qcfg_list, layer)
            variants = [select_variant(tiles, nat.default_variant())]
        else:  # every compiled variant that has a tile body for each qcfg of the layer
            variants = [v for v in nat.production_variants(None) if all(nat.variant_supports(v, q) for q in qcfg_list)]
        names = nat.list_variants()
        result["variants"][layer] = variants
        parsed = load_workload(wl)[f"layer-{layer}"]
        for gg in ("gate_up", "down"):
            inp = build_layer_inputs(parsed[gg])
            rows = []
            base_ms = None
            if not args.no_baseline:
                fp = [(torch.empty(max(s.M, 1), s.K, dtype=torch.float16, device="cuda").uniform_(-1, 1),
                       torch.empty(s.N, s.K, dtype=torch.float16, device="cuda").uniform_(-1, 1)) for s in parsed[gg]]

                def base():
                    for a, b in fp:
                        torch.matmul(a, b.t())
                base_ms = time_launches(base, warmup=3, iters=max(5, args.iters // 5))["median_ms"]
                rows.append({"kernel_name": "torch.matmul_fp16_per_problem", "avg_time": base_ms,
                             "TFLOPS": inp.flops / (base_ms * 1e-3) / 1e12, "speedup": 1.0})
                del fp
            for v in variants:
                g = GroupGemm(inp.problems, variant=v)
                if args.mode == "check":
                    g.launch()
                    torch.cuda.synchronize()
                    check_sampled(inp.problems)
                    print(f"  CHECK {gg} {names[v]}: OK")
                t = time_launches(g.launch, warmup=min(30, args.iters), iters=args.iters)
                tf = inp.flops / (t["median_ms"] * 1e-3) / 1e12
                rows.append({"kernel_name": names[v].split()[1], "avg_time": t["median_ms"], "TFLOPS": tf,
                             "speedup": (base_ms / t["median_ms"]) if base_ms else float("nan")})
                print(f"  {gg} {names[v].split()[1]}: {t['median_ms']:.4f} ms  {tf:.1f} TFLOP/s")
            bench_save = f"{CUR_DIR}/out/bench/{args.model}-{args.dataset}-{args.bs}{suffix.replace('.json', '')}"
            write_csv(f"{bench_save}-layer-{layer}-{gg}.csv", rows)
            result["csv"].append(f"{bench_save}-layer-{layer}-{gg}.csv")
            del inp
            torch.cuda.empty_cache()
        print(f"Layer {layer} completed! Results saved to: {bench_save}")
    return result


def cpu_plumbing(args, trace, layers, wl_kw, workload_path, suffix):
    """BASELINE configs[0]: the workload plumbing plus the reference's torch CPU matmul path (fp16,
    one torch.matmul per problem) timed on the host. Nothing here runs or stands in for the HIP
    kernels; it is the baseline the GPU numbers are reported against."""
    import time

    import torch

    from mxmoe_amd.harness import write_csv

    out = []
    for layer in layers:
        wl = generate_workload_from_trace(trace, args.bs, layer, **wl_kw)
        save_workload(wl, workload_path)
        print(f"Save generated workloads to `{workload_path}`")
        parsed = load_workload(wl)[f"layer-{layer}"]
        g = torch.Generator().manual_seed(42)
        for gg in ("gate_up", "down"):
            fp = [((torch.rand(max(s.M, 1), s.K, generator=g) * 2 - 1).half(),
                   (torch.rand(s.N, s.K, generator=g) * 2 - 1).half()) for s in parsed[gg]]
            flops = sum(2.0 * s.M * s.N * s.K for s in parsed[gg])
            for a, b in fp[:2]:
                torch.matmul(a, b.t())  # warm-up
            t0 = time.perf_counter()
            for a, b in fp:
                torch.matmul(a, b.t())
            ms = (time.perf_counter() - t0) * 1e3
            row = {"kernel_name": "torch.matmul_fp16_per_problem_cpu", "avg_time": ms,
                   "TFLOPS": flops / (ms * 1e-3) / 1e12, "speedup": 1.0}
            bench_save = f"{CUR_DIR}/out/bench/{args.model}-{args.dataset}-{args.bs}{suffix.replace('.json', '')}"
            write_csv(f"{bench_save}-layer-{layer}-{gg}-cpu.csv", [row])
            print(f"  {gg} cpu torch.matmul fp16: {ms:.2f} ms  {row['TFLOPS'] * 1e3:.2f} GFLOP/s "
                  f"({len(parsed[gg])} problems, {torch.get_num_threads()} threads)")
            out.append((layer, gg, len(parsed[gg]), ms))
    return out


if __name__ == "__main__":
    main()
