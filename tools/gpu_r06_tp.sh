#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r06_traffic.sh && bash tools/gpu_r06_plan2.sh plan2
