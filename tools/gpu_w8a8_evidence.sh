#!/bin/bash
# GPU box: w8a8 evidence for the current planner — PMC counter passes (gate_up, down; AUTO variant)
# and bench.py --config w8a8 with its rocprofv3 kernel-trace stats; raw per-dispatch CSVs are
# deleted after summarising (gpurun copies back at most 64 MiB).  usage: bash tools/gpu_w8a8_evidence.sh <tag> [ggs]
set -o pipefail
TAG=${1:-w8a8}
GGS=${2:-"gate_up down"}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for gg in $GGS; do
  timeout -k 10 900 bash tools/pmc_sweep.sh ${TAG}_$gg --cfg w8a8 --gg $gg --variants auto --iters 20 > gpurun_out/pmc_${TAG}_$gg.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_${TAG}_$gg/p*/
  grep -A 30 "gg_v2_kernel" gpurun_out/pmc_${TAG}_$gg.txt || true
done
timeout -k 10 900 bash tools/gpu_bench_profile.sh ${TAG}_bench --config w8a8 > gpurun_out/bench_profile_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_profile_${TAG}.log; exit 1; }
rm -f gpurun_out/prof_${TAG}_bench/run_kernel_trace.csv
head -3 gpurun_out/prof_${TAG}_bench/run_kernel_stats.csv | cut -c1-200
