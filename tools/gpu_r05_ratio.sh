#!/bin/bash
# GPU box, round 5: layer calls and dense 8192^3 on the product library's AUTO kernel, same process
# per config (no trace build: the per-tile cost of the layer against the dense mainloop rate)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05/${1:-ratio}
mkdir -p $OUT
for cfg in w8a8 fp16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants auto --iters 30 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants auto --iters 20 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done
cut -c1-200 $OUT/kbench.jsonl
