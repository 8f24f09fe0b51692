#!/bin/bash
# GPU box: where the persistent v2p variant loses — dense, shared-only and routed-only calls vs v2s.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_v2p_diag.jsonl
: > $OUT
for cfg in w8a8 fp16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 8,21 --iters 10 --rounds 3 >> $OUT 2>>gpurun_out/kbench_v2p_diag.err || exit 1
  for only in shared routed; do
    for gg in gate_up down; do
      timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --only $only --variants 8,21 --iters 20 --rounds 3 >> $OUT 2>>gpurun_out/kbench_v2p_diag.err || exit 1
    done
  done
done
cat $OUT
