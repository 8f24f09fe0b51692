#!/bin/bash
# GPU box (product library): AUTO vs v2x (8) vs wo3 (9) on weight-only layer-11 calls over batch sizes.
# usage: tools/gpu_wo3_auto.sh TAG "BATCHES" [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; BSS=${2:-"128 256 1024 4096"}; CFGS=${3:-"w4a16 w4a16c w8a16 w2a16"}
mkdir -p gpurun_out
OUT=gpurun_out/wo3auto_$TAG.jsonl
: > $OUT
for cfg in $CFGS; do
  for bs in $BSS; do
    for gg in gate_up down; do
      timeout -k 10 200 python tools/kbench.py --cfg $cfg --bs $bs --gg $gg --variants auto,8,9 --iters 30 --rounds 6 >> $OUT 2>>gpurun_out/wo3auto_$TAG.err || exit 1
    done
  done
done
python - $OUT <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    print(r["cfg"], r["gg"], r.get("bs", ""), r["spec"], r["variant"], r["median_ms"], r["tflops"], r["gbs"], r["tiles"])
PY
