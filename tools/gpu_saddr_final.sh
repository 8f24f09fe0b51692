#!/bin/bash
# GPU box: saddr-form LDS-DMA addresses in the production v2s (8) / v2s3 (17) vs their addr64 copies
# (21 / 22): round-robin A/B on every layer-11 call, then the whole round check.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_saddr2.jsonl
: > $OUT
for cfg in fp16 w8a8 mixed bf16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg gate_up --variants 8,21,17,22 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_saddr2.err || exit 1
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg down --variants 17,22 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_saddr2.err || exit 1
done
cut -c1-120 $OUT
bash tools/gpu_round_check.sh r02s
