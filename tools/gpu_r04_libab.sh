#!/bin/bash
# GPU box: A/B of two builds of the same variant in alternating processes (for a change that has
# no ABL bit): usage tools/gpu_r04_libab.sh TAG LIB_A LIB_B VARIANT "cfgs" "bss"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; LA=$2; LB=$3; V=$4; CFGS=$5; BSS=$6
OUT=gpurun_out/r04/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for lib in $LA $LB; do
    for bs in $BSS; do
      for cfg in $CFGS; do
        for gg in gate_up down; do
          MXMOE_GG_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants $V --iters 40 --rounds 8 \
            | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
        done
      done
    done
  done
done
echo done
