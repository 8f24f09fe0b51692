#!/bin/bash
# GPU box (fast lab): wo3 (variant 6) with every problem split into S K slices (MXMOE_GG_SPLITK_ALL)
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
OUT=gpurun_out/wo3split_$1.jsonl
: > $OUT
for bs in ${2:-"512 2048"}; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg w4a16 --bs $bs --gg $gg --variants 4,6,6@MXMOE_GG_SPLITK_ALL=2,6@MXMOE_GG_SPLITK_ALL=3,6@MXMOE_GG_SPLITK_ALL=4 --iters 30 --rounds 6 >> $OUT 2>>gpurun_out/wo3split_$1.err || exit 1
  done
done
python - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["gg"], r["bs"], r["spec"], r["median_ms"], r["tflops"], r["gbs"], r["tiles"], r["grid"])
PY
