#!/bin/bash
# GPU box: the whole -m gpu suite, smoke(), then bench.py + rocprofv3 kernel stats (tools/gpu_bench_profile.sh).
# usage: bash tools/gpu_round_check.sh <tag>
set -o pipefail
TAG=${1:-r02}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
bash tools/gpu_bench_profile.sh $TAG
