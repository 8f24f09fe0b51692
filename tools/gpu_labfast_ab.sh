#!/bin/bash
# GPU box: fast-lab experiments (python -m mxmoe_amd.build --lab-fast: fp16 / w8a8 bodies only).
# Parity screen of the listed variants, then round-robin A/B (tools/kbench.py) on the layer-11 calls
# and dense 8192^3. usage: tools/gpu_labfast_ab.sh TAG "VARIANTS" [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; VARS=$2; CFGS=${3:-"w8a8 fp16"}
mkdir -p gpurun_out
OUT=gpurun_out/labfast_$TAG.jsonl
: > $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants $VARS --cases fp16,w8a8 > gpurun_out/labfast_parity_$TAG.jsonl 2>gpurun_out/labfast_parity_$TAG.err || { tail -5 gpurun_out/labfast_parity_$TAG.err; grep '"ok": false' gpurun_out/labfast_parity_$TAG.jsonl; exit 1; }
echo parity ok
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $VARS --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/labfast_$TAG.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants $VARS --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/labfast_$TAG.err || exit 1
done
cut -c1-400 $OUT
