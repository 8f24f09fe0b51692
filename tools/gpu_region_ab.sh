#!/bin/bash
# GPU box: parity of the region planner, kbench A/B of XCD regions on / off, PMC traffic both ways.
# usage: bash tools/gpu_region_ab.sh <tag>
set -o pipefail
TAG=${1:-region}
cd $GRAFT_REPO_ROOT
# the planner A/B switches (MXMOE_GG_BAND / _REGION / ...) exist only in the lab library (-DMXMOE_LAB)
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "build the lab library first: python -m mxmoe_amd.build --lab"; exit 1; }
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
for cfg in fp16 w8a8 mixed; do
  for gg in gate_up down; do
    timeout -k 10 120 python tools/kbench.py --cfg $cfg --gg $gg --variants "auto,auto@MXMOE_GG_REGION=0" --iters 40 --rounds 8 >> gpurun_out/$TAG/kbench_region_ab.jsonl || exit 1
  done
done
cat gpurun_out/$TAG/kbench_region_ab.jsonl
PMC_OUT=gpurun_out/$TAG/pmc_on timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 mixed > gpurun_out/$TAG/pmc_on.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_on.log; exit 1; }
MXMOE_GG_REGION=0 PMC_OUT=gpurun_out/$TAG/pmc_off timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 > gpurun_out/$TAG/pmc_off.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_off.log; exit 1; }
grep hbm_bytes_per_step gpurun_out/$TAG/pmc_on/pmc_traffic.json gpurun_out/$TAG/pmc_off/pmc_traffic.json
