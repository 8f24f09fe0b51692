#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r06_plan.sh plan && bash tools/gpu_r06_perf.sh perf
