#!/bin/bash
# GPU box: w8a8 evidence for the current planner — PMC counter passes (gate_up, down; AUTO variant)
# and bench.py --config w8a8 with its rocprofv3 kernel-trace stats.  usage: bash tools/gpu_w8a8_evidence.sh <tag>
set -o pipefail
TAG=${1:-w8a8}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash tools/pmc_sweep.sh ${TAG}_gate_up --cfg w8a8 --gg gate_up --variants auto --iters 20 > gpurun_out/pmc_${TAG}_gate_up.txt 2>&1 || exit 1
timeout -k 10 900 bash tools/pmc_sweep.sh ${TAG}_down --cfg w8a8 --gg down --variants auto --iters 20 > gpurun_out/pmc_${TAG}_down.txt 2>&1 || exit 1
cat gpurun_out/pmc_${TAG}_gate_up.txt | grep -v "^W\|^E\|^I"
timeout -k 10 900 bash tools/gpu_bench_profile.sh ${TAG}_bench --config w8a8 > gpurun_out/bench_profile_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_profile_${TAG}.log; exit 1; }
head -3 gpurun_out/prof_${TAG}_bench/*/*kernel_stats.csv gpurun_out/prof_${TAG}_bench/*kernel_stats.csv 2>/dev/null | cut -c1-200
