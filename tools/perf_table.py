"""Measure the MI355X kernel performance table (reference schema, mxmoe_amd/perf_table.py).

python tools/perf_table.py [--out profiles/r01/performance_table_mi355x.json] [--qcfgs fp16,w8a8_g-1_sym,...]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mxmoe_amd import perf_table  # noqa: E402
from mxmoe_amd.perf_table import MEASURED_QCFG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "mxmoe_amd", "workloads", "performance_table_mi355x.json"))
    ap.add_argument("--qcfgs", default=",".join(MEASURED_QCFG))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--merge", action="store_true", help="keep the other qcfgs of an existing --out file")
    args = ap.parse_args()
    table = perf_table.measure([q for q in args.qcfgs.split(",") if q], iters=args.iters,
                               log=lambda m: print(m, file=sys.stderr, flush=True))
    perf_table.dump(table, args.out, merge=args.merge)
    print(args.out)


if __name__ == "__main__":
    main()
