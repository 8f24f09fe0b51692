#!/bin/bash
# GPU box, round 4: HBM counter bytes (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.sh) for the
# fp16 headline and the small-batch w4a16 + w8a8 calls, then bench.py at the driver's 5-step warm-up.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04/pmc
PMC_OUT=gpurun_out/r04/pmc/fp16 bash tools/pmc_traffic.sh fp16 > gpurun_out/r04/pmc/fp16.log 2>&1 || { tail -20 gpurun_out/r04/pmc/fp16.log; exit 1; }
PMC_OUT=gpurun_out/r04/pmc/bs512 KB_ARGS="--bs 512" bash tools/pmc_traffic.sh w4a16_w8a8 > gpurun_out/r04/pmc/bs512.log 2>&1 || { tail -20 gpurun_out/r04/pmc/bs512.log; exit 1; }
find gpurun_out/r04/pmc -name "*.csv" -size +2M -delete
timeout -k 10 400 python bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-scaling-sim > gpurun_out/r04/pmc/bench_w5.json 2> gpurun_out/r04/pmc/bench_w5.err || exit 1
cat gpurun_out/r04/pmc/fp16/pmc_traffic.json gpurun_out/r04/pmc/bs512/pmc_traffic.json
