#!/bin/bash
# GPU box: PMC traffic of the product AUTO variant, then the lab library's v2x twin planned with
# the given placement env (MXMOE_GG_* knobs), then a round-robin time A/B of the two placements.
# usage: tools/gpu_traffic_ab.sh TAG LABVAR "ENV1 ENV2 ..." [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; LV=$2; ENVS=$3; CFGS=${4:-"fp16 w8a8"}
OUT=gpurun_out/traffic_$TAG
mkdir -p $OUT
PMC_OUT=$OUT/auto timeout -k 10 600 bash tools/pmc_traffic.sh $CFGS > $OUT/auto.log 2>&1 || { tail -20 $OUT/auto.log; exit 1; }
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VARS=$LV
for e in $ENVS; do
  PMC_OUT=$OUT/$e KB_ARGS="--variants $LV@$e" timeout -k 10 600 bash tools/pmc_traffic.sh $CFGS > $OUT/$e.log 2>&1 || { tail -20 $OUT/$e.log; exit 1; }
  VARS="$VARS,$LV@$e"
done
find $OUT -name "*.csv" -delete
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $VARS --iters 40 --rounds 10 >> $OUT/time.jsonl 2>>$OUT/time.err || exit 1
  done
done
grep -h hbm_bytes_per_step $OUT/*/pmc_traffic.json
