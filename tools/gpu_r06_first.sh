#!/bin/bash
# GPU box, round 6, first call: the round-5 tree's bench line + layer / dense ratio (gpu_r06_base.sh),
# then the v4d / XCD-packing lab screen (gpu_r06_v4.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r06_base.sh base && bash tools/gpu_r06_v4.sh v4a
