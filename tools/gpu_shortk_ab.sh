#!/bin/bash
# GPU box: long-K calls (fp16 / bf16 gate_up, K = 4096 B = 32 stages) on v2s (8) vs v2s3 (17),
# round-robin, two independent runs each: does the short-K threshold (24 stages) leave speed behind?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_shortk.jsonl
: > $OUT
for rep in 1 2; do
  for cfg in fp16 bf16; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg gate_up --variants 8,17 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_shortk.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg fp16 --gg gate_up --only shared --variants 8,17 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_shortk.err || exit 1
  timeout -k 10 200 python tools/kbench.py --cfg fp16 --gg gate_up --only routed --variants 8,17 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_shortk.err || exit 1
done
cat $OUT
