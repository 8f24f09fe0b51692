#!/bin/bash
# GPU box, round 6: tile timelines of the small-batch calls on the product loop (lab abl_wo3_pch_trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-wotrace}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
for gg in gate_up down; do
  timeout -k 10 120 python tools/tile_trace.py --cfg w4a16_w8a8 --gg $gg --bs 512 --variant-name abl_wo3_pch_trace --dump $OUT/trace_$gg.npy >> $OUT/trace.jsonl 2>> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
done
cat $OUT/trace.jsonl
