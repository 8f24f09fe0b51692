"""Parity screen of a lab weight-only loop option against the lab copy of the product loop (GPU box).

MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so python tools/wo_lab_parity.py --base x_wo3 --test x_wo3_pch

Weight-only problems (per-channel and g128, sym / asym, split-K long K, a w8a8 problem beside them):
the test variant's outputs must equal the base variant's bit for bit (same arithmetic, same order),
and both must sit within the fp16 tolerance of the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.groupgemm import W8A8, QParams, group_gemm  # noqa: E402
from tests._util import HostProblem, assert_f16_close  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", default="x_wo3")
    ap.add_argument("--test", default="x_wo3_pch")
    args = ap.parse_args()
    names = [ln.split()[1] for ln in nat.list_variants()]
    vb, vt = names.index(args.base), names.index(args.test)
    shapes = [(1, 128, 256), (17, 256, 128), (35, 256, 2048), (64, 8, 1024), (130, 136, 384), (257, 264, 512),
              (40, 2816, 2048), (48, 2048, 5632), (512, 512, 1408)]
    qs = [QParams(16, 4, -1, False), QParams(16, 4, -1, True), QParams(16, 4, 128, False), QParams(16, 8, -1, False)]
    bad = 0
    for q in qs:
        for mix in ((False,) if q.w_bits == 8 else (False, True)):  # (fast lab: no w8a16 + w8a8 build)
            specs = [(M, N, K if q.gsize == -1 or K % q.gsize == 0 else 256, q) for M, N, K in shapes]
            if mix:
                specs.append((48, 256, 512, W8A8))
            outs = []
            for v in (vb, vt):
                hps = [HostProblem(M, N, K, qq, seed=500 + i, device="cuda") for i, (M, N, K, qq) in enumerate(specs)]
                group_gemm([h.problem for h in hps], variant=v)
                torch.cuda.synchronize()
                outs.append(hps)
            same = all(torch.equal(a.problem.C.view(torch.int16), b.problem.C.view(torch.int16))
                       for a, b in zip(*outs))
            ok = True
            try:
                for h in outs[1]:
                    if h.M:
                        assert_f16_close(h.result(), h.expected(), h.K)
            except AssertionError as e:
                ok = False
                print(str(e)[:200], file=sys.stderr)
            bad += (not same) or (not ok)
            print(json.dumps({"q": q.qcfg, "mix_w8a8": mix, "bit_identical_to_base": same, "oracle_ok": ok}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
