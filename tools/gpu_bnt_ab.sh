#!/bin/bash
# GPU box: parity of the nt-B variants (v2s_bnt = 21, v2s3_bnt = 22), then round-robin A/B
# against v2s (8) / v2s3 (17) on the layer-11 calls and dense 8192^3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_bnt.log 2>&1 || { tail -40 gpurun_out/pytest_bnt.log; exit 1; }
tail -2 gpurun_out/pytest_bnt.log
OUT=gpurun_out/kbench_bnt.jsonl
: > $OUT
for cfg in w8a8 fp16 mixed; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,21,22 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_bnt.err || exit 1
    tail -1 $OUT | cut -c1-400
  done
done
for cfg in w8a8 fp16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 8,17,21,22 --iters 10 --rounds 3 >> $OUT 2>>gpurun_out/kbench_bnt.err || exit 1
done
cat $OUT
