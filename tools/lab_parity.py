"""Parity screen of the lab library's mainloop experiments (libmxmoe_gg_lab.so, GPU box).

MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so python tools/lab_parity.py [--variants 2,3]

Runs every non-ablation lab variant (or the listed ones) over the edge shapes of
tests/test_gg_gpu.py (fp16 / w8a8 / w4a4, a w8a8 + w4a4 fused launch, K tails inside a stage,
long K) against the C oracle: bit-exact for the integer paths, the fp16 tolerance otherwise.
Prints one JSON line per (variant, case) and exits non-zero on any mismatch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mxmoe_amd import _native as nat  # noqa: E402
from mxmoe_amd.groupgemm import FP16, W4A4, W8A8, QParams, group_gemm  # noqa: E402
from tests._util import HostProblem, assert_f16_close, exact_compare  # noqa: E402


def cases():
    edge = [(1, 128, 256), (17, 256, 128), (130, 128, 384), (257, 136, 512), (64, 8, 1024), (300, 520, 512),
            (513, 264, 256), (600, 512, 4096)]
    for q, name in ((FP16, "fp16"), (W8A8, "w8a8"), (W4A4, "w4a4")):
        yield name + "_edge", [(M, N, K, q) for M, N, K in edge]
        bits = 16 if not q.is_quant else q.a_bits
        yield name + "_ktail", [(70 + 61 * t, 128 + 8 * t, (128 * 8 // bits) * (3 + 5 * t) + (128 // bits) * t, q)
                                for t in range(1, 8)]
    yield "mixed", [(300, 256, 256, W8A8), (0, 256, 256, W4A4), (129, 384, 512, W4A4), (513, 256, 1280, W8A8),
                    (5, 128, 64, W4A4), (384, 512, 2048, W8A8), (512, 768, 4096, W4A4)]
    # weight-only w4a16 (the lab build compiles the 4-bit body only): edge shapes of
    # tests/test_weightonly_gpu.py plus small-batch expert shapes (long K, many scale groups)
    for g in (-1, 128):
        for sym in (True, False):
            q = QParams(16, 4, g, sym)
            yield f"w4a16_g{g}_{'sym' if sym else 'asym'}", [
                (M, N, K, q) for M, N, K in [(1, 128, 256), (17, 256, 128 if g == -1 else 256), (130, 136, 384),
                                             (257, 264, 512), (513, 512, 1408), (64, 8, 1024), (34, 2816, 2048),
                                             (41, 2048, 1408), (96, 512, 640)]]
    # the small-batch pairing (w4a16 + w8a8 in one launch: wo3's QM = 10 build)
    yield "w4a16w8a8", [(34, 2816, 2048, QParams(16, 4, -1, False)), (41, 2048, 1408, QParams(16, 4, 128, False)),
                        (57, 256, 512, W8A8), (3, 128, 256, QParams(16, 4, 128, True)), (130, 384, 1024, W8A8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="")
    ap.add_argument("--cases", default="", help="comma list of case-name prefixes (fast lab: fp16,w8a8)")
    args = ap.parse_args()
    prefixes = tuple(c for c in args.cases.split(",") if c)
    names = {int(ln.split()[0]): ln.split()[1] for ln in nat.list_variants()}
    vs = [int(v) for v in args.variants.split(",")] if args.variants else \
        [i for i, n in names.items() if not n.startswith("abl_")]
    bad = 0
    for v in vs:
        for case, specs in cases():
            if prefixes and not case.startswith(prefixes):
                continue
            hps = [HostProblem(M, N, K, q, seed=31 + i, device="cuda") for i, (M, N, K, q) in enumerate(specs)]
            group_gemm([h.problem for h in hps], variant=v)
            torch.cuda.synchronize()
            worst = 0
            for hp in hps:
                out, ref = hp.result(), hp.expected()
                if exact_compare(hp.q):
                    worst = max(worst, int(np.count_nonzero(out.view(np.uint16) != ref.view(np.uint16))))
                else:
                    try:
                        assert_f16_close(out, ref, hp.K)
                    except AssertionError:
                        worst = max(worst, 1)
            bad += worst > 0
            print(json.dumps({"variant": v, "name": names[v], "case": case, "ok": worst == 0, "mismatch": worst}),
                  flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
