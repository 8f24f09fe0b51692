#!/bin/bash
# GPU box: bench.py + rocprofv3 kernel stats for the quantised headline configs (one after another);
# per-dispatch trace CSVs deleted (gpurun copies back at most 64 MiB).
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-mixed w4a4 ds2_mixed}; do
  timeout -k 10 600 bash tools/gpu_bench_profile.sh cfg_$c --config $c --extras "" --no-scaling-sim > gpurun_out/cfg_$c.log 2>&1 || { tail -20 gpurun_out/cfg_$c.log; exit 1; }
  rm -f gpurun_out/prof_cfg_$c/run_kernel_trace.csv
  head -c 300 gpurun_out/bench_cfg_$c.json; echo
done
