#!/bin/bash
# GPU box: the whole -m gpu suite, then the PMC traffic passes of the default build.
set -o pipefail
TAG=${1:-suite}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PMC_OUT=$OUT/pmc timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 mixed > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
find $OUT/pmc -name "*.csv" -delete
grep hbm_bytes_per_step $OUT/pmc/pmc_traffic.json
