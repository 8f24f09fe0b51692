#!/bin/bash
# GPU box: B-before-A DMA issue order (variant 21, v2s_saddr): parity, then round-robin A/B vs v2s (8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_saddr.log 2>&1 || { tail -40 gpurun_out/pytest_saddr.log; exit 1; }
tail -1 gpurun_out/pytest_saddr.log
OUT=gpurun_out/kbench_saddr.jsonl
: > $OUT
for rep in 1 2; do
  for cfg in fp16 bf16 w8a8; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg gate_up --variants 8,21 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_saddr.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg fp16 --dense 8192,8192,8192 --variants 8,21 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_saddr.err || exit 1
done
cut -c1-170 $OUT
