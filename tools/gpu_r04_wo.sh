#!/bin/bash
# GPU box, round 4: small-batch weight-only tile (wo3) A/B in the fast lab build: parity screen of
# the correct variants, then round-robin kbench over the bs 512 / 128 weight-only calls.
# usage: tools/gpu_r04_wo.sh TAG "CORRECT_VARIANTS" "ALL_VARIANTS" [cfgs] [bss]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "missing $MXMOE_GG_LIB"; exit 1; }
TAG=$1; OK=$2; VARS=$3; CFGS=${4:-"w4a16_w8a8 w4a16 w4a16c"}; BSS=${5:-"512 128"}
OUT=gpurun_out/r04/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants $OK --cases w4a16 > $OUT/parity.jsonl 2>$OUT/parity.err || { tail -5 $OUT/parity.err; grep '"ok": false' $OUT/parity.jsonl | head; exit 1; }
echo parity ok
for bs in $BSS; do
  for cfg in $CFGS; do
    for gg in gate_up down; do
      timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants $VARS --iters 40 --rounds 8 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
    done
  done
done
cut -c1-200 $OUT/kbench.jsonl
exit 0
