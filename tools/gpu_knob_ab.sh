#!/bin/bash
# GPU box: round-robin A/B of planner switches on the lab v2x twin.
# usage: tools/gpu_knob_ab.sh TAG LABVAR "ENV1 ENV2 ..." "cfg:bs ..."
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; LV=$2; ENVS=$3; CASES=$4
OUT=gpurun_out/knob_$TAG.jsonl; mkdir -p gpurun_out; : > $OUT
VARS=$LV; for e in $ENVS; do VARS="$VARS,$LV@$e"; done
for cb in $CASES; do
  cfg=${cb%%:*}; bs=${cb#*:}
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --bs $bs --gg $gg --variants $VARS --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/knob_$TAG.err || exit 1
  done
done
cut -c1-120 $OUT
