#!/bin/bash
# Round GPU job: bench.py (JSON line) + rocprofv3 kernel-trace stats of the same command.
# usage: bash tools/gpu_bench_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p $OUT
cd $REPO
timeout -k 10 400 python bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
cat $OUT/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python3 bench.py --no-cpu-baseline --no-scaling-sim --extras "" "$@" > $OUT/bench_prof_$TAG.json 2> $OUT/prof_$TAG.err || exit $?
find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs cat
