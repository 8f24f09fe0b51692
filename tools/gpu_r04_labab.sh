#!/bin/bash
# GPU box, round 4: fast-lab A/B (parity screen, round-robin kbench on the layer-11 calls + dense
# 8192^3) then tile timelines of the traced builds. usage: tools/gpu_r04_labab.sh TAG "VARIANTS" "TRACE_NAMES" [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; VARS=$2; TRACES=$3; CFGS=${4:-"w8a8 fp16"}
OUT=gpurun_out/r04/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants $VARS --cases fp16,w8a8 > $OUT/parity.jsonl 2>$OUT/parity.err || { tail -5 $OUT/parity.err; grep '"ok": false' $OUT/parity.jsonl | head; exit 1; }
echo parity ok
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $VARS --iters 40 --rounds 8 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants $VARS --iters 20 --rounds 4 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done
cut -c1-300 $OUT/kbench.jsonl
for name in $TRACES; do
  for cfg in $CFGS; do
    for gg in gate_up down; do
      timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --gg $gg --variant-name $name >> $OUT/trace.jsonl 2>>$OUT/trace.err || exit 1
    done
  done
done
[ -n "$TRACES" ] && cut -c1-600 $OUT/trace.jsonl
exit 0
