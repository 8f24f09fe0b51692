#!/bin/bash
# GPU box: the low-B-reuse AUTO rule (gate_up calls now on v2s3) — round-robin A/B of AUTO vs the
# old choice v2s (8) per config, then the whole round check (tests, smoke, bench + rocprof).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_reuse.jsonl
: > $OUT
for cfg in fp16 bf16 ds2_mixed; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg gate_up --variants auto,8 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_reuse.err || exit 1
done
tail -6 $OUT
bash tools/gpu_round_check.sh r02h
