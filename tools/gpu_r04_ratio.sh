#!/bin/bash
# GPU box, round 4: the headline kernel's layer / dense ratio (VERDICT r03 item 1 metric): product
# v2x (variant 1) on the w8a8 / fp16 bs 8192 calls and on dense 8192^3, plus the lab trace build's
# tile timeline of the w8a8 / fp16 gate_up calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04/ratio; mkdir -p $OUT
for cfg in w8a8 fp16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 1 --iters 40 --rounds 4 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 1 --iters 20 --rounds 4 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --gg gate_up --variant-name abl_v2x_trace >> $OUT/trace.jsonl 2>>$OUT/trace.err || exit 1
done
cut -c1-300 $OUT/kbench.jsonl; cut -c1-700 $OUT/trace.jsonl
