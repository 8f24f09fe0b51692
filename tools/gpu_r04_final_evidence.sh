#!/bin/bash
# GPU box, round 4: bench + rocprofv3 kernel stats of the small-batch scheme as the main config, and
# PMC traffic of the w8a8 / w4a4 / mixed headline extras (tools/pmc_traffic.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04/final; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config w4a16_w8a8_bs512 --extras "" --no-cpu-baseline --no-scaling-sim > $OUT/bench_bs512.json 2> $OUT/bench_bs512.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bs512 -o run -- \
  python3 bench.py --config w4a16_w8a8_bs512 --extras "" --no-cpu-baseline --no-scaling-sim > $OUT/bench_bs512_prof.json 2> $OUT/prof_bs512.err || exit 1
PMC_OUT=$OUT/pmc bash tools/pmc_traffic.sh w8a8 w4a4 mixed > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
find $OUT -name "*counter_collection.csv" -delete
cat $OUT/bench_bs512.json; find $OUT/prof_bs512 -name "*kernel_stats.csv" | head -1 | xargs head -4; cat $OUT/pmc/pmc_traffic.json | head -40
