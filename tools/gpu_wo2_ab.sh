#!/bin/bash
# GPU box: weight-only tile with 2 / 3 workgroups per CU (fast lab: x_wo2_64 / x_wo3_64) against the
# v2x weight-only body (x_v2x_wo): parity screen, then round-robin A/B over batch sizes.
# usage: tools/gpu_wo2_ab.sh TAG "VARIANTS" "BATCHES" [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; VARS=$2; BSS=${3:-"128 512 2048"}; CFGS=${4:-"w4a16 w4a16c"}
mkdir -p gpurun_out
OUT=gpurun_out/wo2_$TAG.jsonl
: > $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants $VARS --cases w4a16 > gpurun_out/wo2_parity_$TAG.jsonl 2>gpurun_out/wo2_parity_$TAG.err || { tail -5 gpurun_out/wo2_parity_$TAG.err; grep '"ok": false' gpurun_out/wo2_parity_$TAG.jsonl; exit 1; }
echo parity ok
for cfg in $CFGS; do
  for bs in $BSS; do
    for gg in gate_up down; do
      timeout -k 10 200 python tools/kbench.py --cfg $cfg --bs $bs --gg $gg --variants $VARS --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/wo2_$TAG.err || exit 1
    done
  done
done
python - $OUT <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    print(r["cfg"], r["gg"], r.get("bs", ""), r["variant"], r["median_ms"], r["tflops"], r["gbs"], r["tiles"])
PY
