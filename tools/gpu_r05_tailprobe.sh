#!/bin/bash
# GPU box, round 5: cost of one tile by class in isolation — dense calls of M = 64 / 128 / 256 rows
# over N = 131072 (512 n-tiles: two rounds of the CUs), K = 2048, on the AUTO kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tailprobe}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
for cfg in fp16 w8a8; do
  for M in 64 128 192 256; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense $M,131072,2048 --variants auto --iters 20 --rounds 3 \
      >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
cut -c1-220 $OUT/kbench.jsonl
