"""Where a spread-mainloop stage spends its cycles (lab library, V2_STAMP variants; GPU box).

MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so python tools/stamps.py --variants 8,9 [--cfg w8a8]

Per (block, wave) the kernel sums s_memtime cycles over its steady K stages: body (loop top to the
last MFMA issued), vm (the stage-end vmcnt(0) wait: this wave's next-stage LDS-DMA not landed yet)
and bar (the workgroup barrier: waiting for the other waves). Prints per-stage medians for the
early (0-3) and late (4-7) waves as JSON lines.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.groupgemm import GroupGemm  # noqa: E402
from mxmoe_amd.harness import build_layer_inputs  # noqa: E402
from mxmoe_amd.workload import QShape, load_workload, qwen2_layer11_workload  # noqa: E402

NBLK = 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="8,9")
    ap.add_argument("--cfg", default="w8a8")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    lib = nat.lib()
    lib.mxmoe_gg_debug_stamps.restype = ctypes.c_int
    lib.mxmoe_gg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    bits = {"fp16": 16, "w8a8": 8}[args.cfg]
    qkw = {} if bits == 16 else dict(qstr="w8a8_g-1_sym")
    cases = {"dense_8192": [QShape([8192, 8192, 8192], bits, bits)],
             "gate_up": load_workload(qwen2_layer11_workload(8192, **qkw))["layer-11"]["gate_up"],
             "down": load_workload(qwen2_layer11_workload(8192, **qkw))["layer-11"]["down"]}
    for name, shapes in cases.items():
        inp = build_layer_inputs(shapes)
        for v in (int(x) for x in args.variants.split(",")):
            gg = GroupGemm(inp.problems, variant=v)
            for _ in range(args.iters):  # settle the clock, then one stamped launch
                gg.launch()
            torch.cuda.synchronize()
            nat.check(lib.mxmoe_gg_debug_stamps(None, 0, 1))
            gg.launch()
            torch.cuda.synchronize()
            buf = np.zeros(NBLK * 8 * 4, dtype=np.uint64)
            nat.check(lib.mxmoe_gg_debug_stamps(buf.ctypes.data, buf.nbytes, 0))
            st = buf.reshape(NBLK, 8, 4).astype(np.float64)
            row = {"case": name, "cfg": args.cfg, "variant": v, "name": nat.list_variants()[v].split()[1]}
            for half, ws in (("early", slice(0, 4)), ("late", slice(4, 8))):
                s = st[:, ws, :].reshape(-1, 4)
                s = s[s[:, 3] > 0]
                if not len(s):
                    continue
                per = s[:, :3] / s[:, 3:4]
                row[half] = {k: round(float(np.median(per[:, i])), 1) for i, k in enumerate(("body", "vm", "bar"))}
                row[half]["stage_cycles"] = round(float(np.median(per.sum(1))), 1)
                row[half]["waves"] = int(len(s))
            print(json.dumps(row), flush=True)
        del inp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
