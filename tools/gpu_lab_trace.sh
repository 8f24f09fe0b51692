#!/bin/bash
# GPU box: tile timelines (tools/tile_trace.py) of lab V2_TRACE variants on the layer-11 calls.
# usage: tools/gpu_lab_trace.sh TAG "variant_name ..." [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; NAMES=$2; CFGS=${3:-"w8a8 fp16"}
mkdir -p gpurun_out
OUT=gpurun_out/trace_$TAG.jsonl
: > $OUT
for name in $NAMES; do
  for cfg in $CFGS; do
    for gg in gate_up down; do
      timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --gg $gg --variant-name $name >> $OUT 2>>gpurun_out/trace_$TAG.err || exit 1
    done
    timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --dense 8192,8192,8192 --variant-name $name >> $OUT 2>>gpurun_out/trace_$TAG.err || exit 1
  done
done
cut -c1-400 $OUT
