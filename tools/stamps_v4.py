"""Where a v4d steady K stage spends its cycles (lab library, OPT & 1 stamp build `abl_v4d_stamp`;
GPU box). Per (block, wave) the kernel sums s_memtime cycles over its steady stages: seg1 (F0's
reads beside F1's deferred rows and the A pieces), seg2 (F0's MFMAs beside F1's reads and the B
pieces), seg3 (F1 rows 0..H), vm (the stage-end vmcnt wait) and bar (the workgroup barrier).
Prints per-stage medians over the waves as JSON lines (the MFMA floor of a stage is 128 x 16 =
2048 cycles at one wave per SIMD).

MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so python tools/stamps_v4.py --variant 2 [--cfg w8a8]
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
    ap.add_argument("--variant", type=int, default=2)
    ap.add_argument("--cfg", default="w8a8")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    lib = nat.lib()
    lib.mxmoe_gg_debug_stamps.restype = ctypes.c_int
    lib.mxmoe_gg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    bits = {"fp16": 16, "w8a8": 8}[args.cfg]
    qkw = {} if bits == 16 else dict(qstr="w8a8_g-1_sym")
    cases = {"dense_8192": [QShape([8192, 8192, 8192], bits, bits)],
             "gate_up": load_workload(qwen2_layer11_workload(8192, **qkw))["layer-11"]["gate_up"]}
    for name, shapes in cases.items():
        inp = build_layer_inputs(shapes)
        gg = GroupGemm(inp.problems, variant=args.variant)
        for _ in range(args.iters):  # settle the clock, then one stamped launch
            gg.launch()
        torch.cuda.synchronize()
        nat.check(lib.mxmoe_gg_debug_stamps(None, 0, 1))
        gg.launch()
        torch.cuda.synchronize()
        buf = np.zeros(NBLK * 8 * 4, dtype=np.uint64)
        nat.check(lib.mxmoe_gg_debug_stamps(buf.ctypes.data, buf.nbytes, 0))
        st = buf.reshape(NBLK, 8, 4).astype(np.float64)
        a, b = st[:, 0:4, :].reshape(-1, 4), st[:, 4:8, :].reshape(-1, 4)
        keep = a[:, 3] > 0
        a, b = a[keep], b[keep]
        per = np.concatenate([a[:, :3], b[:, :2]], axis=1) / a[:, 3:4]
        row = {"case": name, "cfg": args.cfg, "variant": args.variant, "name": nat.list_variants()[args.variant].split()[1],
               "waves": int(len(per))}
        row.update({k: round(float(np.median(per[:, i])), 1) for i, k in enumerate(("seg1", "seg2", "seg3", "vm", "bar"))})
        row["stage_cycles"] = round(float(np.median(per.sum(1))), 1)
        row["mfma_floor"] = 2048
        print(json.dumps(row), flush=True)
        del inp, gg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
