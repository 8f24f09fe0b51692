#!/bin/bash
# GPU box: fp8 E4M3 / bf16 parity tests, their perf-table rows, and their bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fp8_bf16_gpu.py tests/test_gg_gpu.py tests/test_cli_gpu.py tests/test_abi.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_f8.log 2>&1 || { tail -40 gpurun_out/pytest_f8.log; exit 1; }
tail -3 gpurun_out/pytest_f8.log
timeout -k 10 300 python tools/perf_table.py --qcfgs w8a8_g-1_sym_E4M3,bf16 --merge --out gpurun_out/performance_table_mi355x.json > gpurun_out/perf_table_f8.log 2>&1 || { tail -20 gpurun_out/perf_table_f8.log; exit 1; }
for c in w8a8_e4m3 bf16 w8a8; do
  timeout -k 10 300 python bench.py --config $c --extras "" --no-scaling-sim --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json
done
