#!/bin/bash
# GPU box: parity of the 32x32-MFMA variants, then round-robin A/B against v2s / v2s3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py tests/test_fp8_bf16_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_m32.log 2>&1 || { tail -40 gpurun_out/pytest_m32.log; exit 1; }
tail -2 gpurun_out/pytest_m32.log
OUT=gpurun_out/kbench_m32.jsonl
: > $OUT
for cfg in w8a8 fp16 bf16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,21,22 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_m32.err || exit 1
  done
done
for cfg in w8a8 fp16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 8,17,21,22 --iters 10 --rounds 3 >> $OUT 2>>gpurun_out/kbench_m32.err || exit 1
done
cat $OUT
