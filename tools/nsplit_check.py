"""Lab check: a layer call planned with and without MXMOE_GG_WO_NSPLIT=1 (second-round tiles run as
two 64 x 128 N halves) must give bit-identical C (same per-element K order). Fast lab library.

MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so python tools/nsplit_check.py --variant 9 [--bs 512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import build_layer_inputs  # noqa: E402
from mxmoe_amd.workload import load_workload, qwen2_layer11_workload, w4a16_w8a8_qconfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, required=True)
    ap.add_argument("--bs", type=int, default=512)
    args = ap.parse_args()
    bad = 0
    for cfg, kw in (("w4a16_w8a8", dict(qconfig=w4a16_w8a8_qconfig())), ("w4a16", dict(qstr="w4a16_g128_asym")),
                    ("w8a16", dict(qstr="w8a16_g-1_asym"))):
        for gg in ("gate_up", "down"):
            inp = build_layer_inputs(load_workload(qwen2_layer11_workload(args.bs, **kw))["layer-11"][gg])
            outs, tiles = [], []
            for knob in ("0", "1"):
                os.environ["MXMOE_GG_WO_NSPLIT"] = knob
                g = GroupGemm(inp.problems, variant=args.variant)
                for p in inp.problems:
                    p.C.zero_()
                g.launch()
                torch.cuda.synchronize()
                outs.append([p.C.clone() for p in inp.problems])
                tiles.append(g.total_tiles)
            same = all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(*outs))
            bad += not same
            print(json.dumps({"cfg": cfg, "gg": gg, "bs": args.bs, "tiles": tiles, "bit_identical": same}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
