#!/bin/bash
# GPU box: full -m gpu suite with the tail-region planner, placement A/B, PMC traffic of the default.
set -o pipefail
TAG=${1:-region3}
cd $GRAFT_REPO_ROOT
# the planner A/B switches (MXMOE_GG_BAND / _REGION / ...) exist only in the lab library (-DMXMOE_LAB)
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "build the lab library first: python -m mxmoe_amd.build --lab"; exit 1; }
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
V="auto,auto@MXMOE_GG_REGION=0,auto@MXMOE_GG_REGION=1"
for cg in "fp16 gate_up" "fp16 down" "w8a8 gate_up" "w8a8 down" "mixed gate_up" "mixed down" "w4a4 gate_up"; do
  set -- $cg
  timeout -k 10 150 python tools/kbench.py --cfg $1 --gg $2 --variants "$V" --iters 60 --rounds 10 >> gpurun_out/$TAG/kbench.jsonl || exit 1
done
cat gpurun_out/$TAG/kbench.jsonl
PMC_OUT=gpurun_out/$TAG/pmc timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 mixed > gpurun_out/$TAG/pmc.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc.log; exit 1; }
grep hbm_bytes_per_step gpurun_out/$TAG/pmc/pmc_traffic.json
