#!/bin/bash
# GPU box, round 6: first run of the round on the round-5 tree: bench.py JSON line + layer / dense
# 8192^3 kernel timings of the AUTO kernels (same process per config)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-base}
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
for cfg in w8a8 fp16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants auto --iters 30 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants auto --iters 20 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done
cut -c1-200 $OUT/kbench.jsonl
