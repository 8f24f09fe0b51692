#!/bin/bash
# GPU box: region placement (tail / head) x sweep rotation per XCD — kbench A/B + traffic of the winner candidates.
set -o pipefail
TAG=${1:-rot}
cd $GRAFT_REPO_ROOT
# the planner A/B switches (MXMOE_GG_BAND / _REGION / ...) exist only in the lab library (-DMXMOE_LAB)
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "build the lab library first: python -m mxmoe_amd.build --lab"; exit 1; }
mkdir -p gpurun_out/$TAG
V="auto,auto@MXMOE_GG_REGION_ROT=1,auto@MXMOE_GG_REGION=1,auto@MXMOE_GG_REGION=1+ROT"
for cg in "fp16 gate_up" "fp16 down" "w8a8 gate_up" "w8a8 down" "mixed gate_up"; do
  set -- $cg
  timeout -k 10 200 python tools/kbench.py --cfg $1 --gg $2 --variants "auto,auto@MXMOE_GG_REGION_ROT=1,auto@MXMOE_GG_REGION=1" --iters 60 --rounds 10 >> gpurun_out/$TAG/kbench.jsonl || exit 1
  MXMOE_GG_REGION=1 timeout -k 10 200 python tools/kbench.py --cfg $1 --gg $2 --variants "auto,auto@MXMOE_GG_REGION_ROT=1" --iters 60 --rounds 10 | sed 's/"spec": "auto/"spec": "head+auto/' >> gpurun_out/$TAG/kbench.jsonl || exit 1
done
cat gpurun_out/$TAG/kbench.jsonl
for mode in "MXMOE_GG_REGION_ROT=1" "MXMOE_GG_REGION=1 MXMOE_GG_REGION_ROT=1"; do
  tagm=$(echo $mode | tr ' =' '__')
  env $mode PMC_OUT=gpurun_out/$TAG/pmc_$tagm timeout -k 10 600 bash tools/pmc_traffic.sh fp16 w8a8 > gpurun_out/$TAG/pmc_$tagm.log 2>&1 || exit 1
  find gpurun_out/$TAG/pmc_$tagm -name "*.csv" -delete
  echo $mode; grep hbm_bytes_per_step gpurun_out/$TAG/pmc_$tagm/pmc_traffic.json
done
