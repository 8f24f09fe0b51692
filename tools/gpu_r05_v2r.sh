#!/bin/bash
# GPU box, round 5: v2r (persistent v2q resolving each tile from one 128-B record) — parity screen,
# tile timelines and a same-process A/B against v2x and v2q (fast lab library)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-v2r}; VS=${2:-"0,8,11,12"}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
timeout -k 10 300 python tools/lab_parity.py --variants ${PAR_VS:-8,11,12} --cases fp16,w8a8 > $OUT/parity.jsonl 2> $OUT/parity.err || { tail -5 $OUT/parity.jsonl; tail -20 $OUT/parity.err; exit 1; }
grep -c '"ok": true' $OUT/parity.jsonl
for name in ${TRACE_NAMES:-abl_v2x_trace abl_v2q_plain_fillall_trace abl_v2r_plain_fillall_trace}; do
  for cfg in w8a8 fp16; do
    for gg in gate_up down; do
      timeout -k 10 120 python tools/tile_trace.py --cfg $cfg --gg $gg --variant-name $name >> $OUT/trace.jsonl 2>>$OUT/trace.err || exit 1
    done
  done
done
unset MXMOE_GG_LIB
bash tools/gpu_r05_labab.sh $TAG $VS "w8a8 fp16" 8192 ${ROUNDS:-8}
