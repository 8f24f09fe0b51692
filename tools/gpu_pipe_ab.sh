#!/bin/bash
# GPU box: parity of the pipelined variants, then kbench A/B against their parents.
set -o pipefail
TAG=${1:-pipe}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py tests/test_fp8_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
for cg in "w8a8 gate_up" "w8a8 down" "fp16 gate_up" "fp16 down" "bf16 gate_up"; do
  set -- $cg
  timeout -k 10 200 python tools/kbench.py --cfg $1 --gg $2 --variants "8,21,17,22" --iters 60 --rounds 10 >> gpurun_out/$TAG/kbench.jsonl || exit 1
done
timeout -k 10 200 python tools/kbench.py --cfg w8a8 --dense 8192,8192,8192 --variants "8,21,17,22" --iters 20 --rounds 5 >> gpurun_out/$TAG/kbench.jsonl || exit 1
timeout -k 10 200 python tools/kbench.py --cfg fp16 --dense 8192,8192,8192 --variants "8,21,17,22" --iters 20 --rounds 5 >> gpurun_out/$TAG/kbench.jsonl || exit 1
cat gpurun_out/$TAG/kbench.jsonl
