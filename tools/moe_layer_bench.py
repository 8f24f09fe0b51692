"""One qwen2_moe layer-11 MoE FFN step at bs=8192 (LP-1 mixed w4a4 + w8a8 qconfig, routed histogram of
the committed workload, random weights) on the device, unfused (silu_mul_quant) against the fused
SiLU epilogue (MXMOE_GG_EPI_SILU_MUL + quant_slots): moe.qwen2_layer_bench — per-stage and step
times, outputs checked bit-identical.

python tools/moe_layer_bench.py [--rounds 4] [--iters 30] > gpurun_out/moe_layer.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mxmoe_amd import moe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--model", default="qwen2_moe", choices=["qwen2_moe", "ds2"])
    args = ap.parse_args()
    r = moe.qwen2_layer_bench(args.rounds, args.iters, model=args.model)
    r["model"] = args.model
    print(json.dumps(r), flush=True)
    if not r["bit_identical"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
