#!/bin/bash
# GPU box: plan_host's tail split, lab v2x twin with and without it (MXMOE_GG_TAIL_SPLIT=0),
# round-robin A/B on the layer-11 calls.  usage: tools/gpu_tailsplit_ab.sh TAG LABVAR [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; LV=$2; CFGS=${3:-"w8a8 fp16 mixed"}
OUT=gpurun_out/tailsplit_$TAG.jsonl
mkdir -p gpurun_out; : > $OUT
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $LV,$LV@MXMOE_GG_TAIL_SPLIT=0 --iters 60 --rounds 15 >> $OUT 2>>gpurun_out/tailsplit_$TAG.err || exit 1
  done
done
cut -c1-120 $OUT
