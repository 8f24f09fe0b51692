#!/bin/bash
# GPU box: tile timelines of the small-batch weight-only calls (lab trace build of v2x)
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
OUT=gpurun_out/trace_wo.jsonl; mkdir -p gpurun_out; : > $OUT
for bs in 512 128; do for gg in gate_up down; do
  timeout -k 10 120 python tools/tile_trace.py --cfg w4a16ga --bs $bs --gg $gg --variant-name abl_v2x_edma_trace >> $OUT 2>>gpurun_out/trace_wo.err || exit 1
done; done
for gg in gate_up down; do
  timeout -k 10 120 python tools/tile_trace.py --cfg fp16 --bs 512 --gg $gg --variant-name abl_v2x_edma_trace >> $OUT 2>>gpurun_out/trace_wo.err || exit 1
done
cat $OUT
