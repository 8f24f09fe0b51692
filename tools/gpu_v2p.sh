#!/bin/bash
# GPU box: the persistent v2p variant — a short smoke, its parity tests, then an A/B against v2s / v2s3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$(python -c "from mxmoe_amd import _native as n; print([l.split()[1] for l in n.list_variants()].index('v2p_256x256_w8_dma_stagger_persistent'))")
echo "v2p variant $V"
timeout -k 10 120 python -u -m pytest tests/test_gg_gpu.py -x -q -m gpu -k "single_qtype and $V" --timeout 60 --timeout-method thread > gpurun_out/pytest_v2p_smoke.log 2>&1 || { tail -30 gpurun_out/pytest_v2p_smoke.log; exit 1; }
:
timeout -k 10 500 python -u -m pytest tests/test_gg_gpu.py tests/test_golden_gpu.py tests/test_fakequant_gpu.py tests/test_fp8_bf16_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_v2p.log 2>&1 || { tail -30 gpurun_out/pytest_v2p.log; exit 1; }
tail -1 gpurun_out/pytest_v2p.log
OUT=gpurun_out/kbench_v2p.jsonl
: > $OUT
for cfg in w8a8 fp16 mixed w4a4 bf16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,$V --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_v2p.err || exit 1
  done
done
cat $OUT
