#!/bin/bash
# GPU box: the per-tile adaptive B ring (variant 21, v2s3a): parity, round-robin A/B against v2s (8)
# and v2s3 (17) on the layer calls and dense 8192^3, then its PMC counter bytes (fp16, w8a8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py tests/test_golden_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_adapt.log 2>&1 || { tail -40 gpurun_out/pytest_adapt.log; exit 1; }
tail -2 gpurun_out/pytest_adapt.log
OUT=gpurun_out/kbench_adapt.jsonl
: > $OUT
for cfg in fp16 w8a8 mixed bf16 ds2_mixed; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,21 --iters 30 --rounds 10 >> $OUT 2>>gpurun_out/kbench_adapt.err || exit 1
  done
done
for cfg in w8a8 fp16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 8,17,21 --iters 10 --rounds 5 >> $OUT 2>>gpurun_out/kbench_adapt.err || exit 1
done
cut -c1-150 $OUT
PMC_OUT=gpurun_out/pmc_adapt KB_ARGS="--variants 21" bash tools/pmc_traffic.sh fp16 w8a8 > gpurun_out/pmc_adapt.log 2>&1 || { tail -20 gpurun_out/pmc_adapt.log; exit 1; }
tail -30 gpurun_out/pmc_adapt.log
