#!/bin/bash
# GPU box: kbench A/B of planner knobs (band height, tail chunk) on the default planner.
set -o pipefail
TAG=${1:-knobs}
cd $GRAFT_REPO_ROOT
# the planner A/B switches (MXMOE_GG_BAND / _REGION / ...) exist only in the lab library (-DMXMOE_LAB)
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
[ -f "$MXMOE_GG_LIB" ] || { echo "build the lab library first: python -m mxmoe_amd.build --lab"; exit 1; }
mkdir -p gpurun_out/$TAG
V="auto,auto@MXMOE_GG_BAND=2,auto@MXMOE_GG_BAND=8,auto@MXMOE_GG_TAIL_CHUNK=8,auto@MXMOE_GG_TAIL_CHUNK=32"
for cg in "fp16 gate_up" "fp16 down" "w8a8 gate_up" "w8a8 down"; do
  set -- $cg
  timeout -k 10 200 python tools/kbench.py --cfg $1 --gg $2 --variants "$V" --iters 60 --rounds 10 >> gpurun_out/$TAG/kbench.jsonl || exit 1
done
cat gpurun_out/$TAG/kbench.jsonl
