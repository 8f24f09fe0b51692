#!/bin/bash
# GPU box: lab parity of the listed variants (incl. the w4a16 cases), then round-robin A/B on the
# small-batch weight-only calls.  usage: tools/gpu_wo_ab.sh TAG "VARIANTS" ["cfg:bs ..."]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; VARS=$2; CASES=${3:-"w4a16ga:512 w4a16:512 w4a16ga:128 w4a16ga:2048"}
OUT=gpurun_out/wo_$TAG.jsonl
mkdir -p gpurun_out; : > $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants $VARS > gpurun_out/wo_parity_$TAG.jsonl 2>gpurun_out/wo_parity_$TAG.err || { tail -5 gpurun_out/wo_parity_$TAG.err; grep '"ok": false' gpurun_out/wo_parity_$TAG.jsonl; exit 1; }
echo parity ok
for cb in $CASES; do
  cfg=${cb%%:*}; bs=${cb#*:}
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --bs $bs --gg $gg --variants $VARS --iters 60 --rounds 15 >> $OUT 2>>gpurun_out/wo_$TAG.err || exit 1
  done
done
cut -c1-140 $OUT
