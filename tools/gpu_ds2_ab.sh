#!/bin/bash
# GPU box: variants on the DeepSeek-V2-Lite mixed layer (short-K down call) and qwen2 mixed.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ds2
for cg in "ds2_mixed gate_up" "ds2_mixed down" "mixed down"; do
  set -- $cg
  timeout -k 10 200 python tools/kbench.py --cfg $1 --gg $2 --variants "auto,7,8,17,3" --iters 60 --rounds 10 >> gpurun_out/ds2/kbench.jsonl || exit 1
done
cat gpurun_out/ds2/kbench.jsonl
