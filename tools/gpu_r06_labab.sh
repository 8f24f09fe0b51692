#!/bin/bash
# GPU box, round 6: same-process round-robin A/B of lab variants (tools/kbench.py on the lab library)
# usage: tools/gpu_r05_labab.sh TAG "variant list" "cfgs" "bss" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VS=$2; CFGS=$3; BSS=$4; R=${5:-10}; GGS=${6:-"gate_up down"}
OUT=gpurun_out/r06/$TAG
mkdir -p $OUT
for bs in $BSS; do
  for cfg in $CFGS; do
    for gg in $GGS; do
      MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so timeout -k 10 240 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs \
        --variants $VS --iters $((4 * R)) --rounds $R >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
    done
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
