#!/bin/bash
# GPU box: PMC traffic of the fp16 / w8a8 step with band heights 2 and 8 (MXMOE_GG_BAND).
set -o pipefail
cd $GRAFT_REPO_ROOT
# the planner A/B switches (MXMOE_GG_BAND / _REGION / ...) exist only in the lab library (-DMXMOE_LAB)
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "build the lab library first: python -m mxmoe_amd.build --lab"; exit 1; }
for b in 2 8; do
  MXMOE_GG_BAND=$b PMC_OUT=gpurun_out/band$b timeout -k 10 600 bash tools/pmc_traffic.sh fp16 w8a8 > gpurun_out/band$b.log 2>&1 || { tail -20 gpurun_out/band$b.log; exit 1; }
  find gpurun_out/band$b -name "*.csv" -delete
  echo band $b; grep hbm_bytes_per_step gpurun_out/band$b/pmc_traffic.json
done
