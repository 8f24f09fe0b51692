#!/bin/bash
# GPU box, round 5 baseline: the -m gpu suite (every product variant at full size), smoke(), bench.py +
# rocprofv3 kernel stats, and counter passes of the w4a4 AUTO kernel (v3) on the bs=8192 calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05a}
OUT=gpurun_out/r05/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --no-cpu-baseline --no-scaling-sim --extras "" > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cat
# w4a4 (v3) counters: MFMA busy, wait split, L2 hit, plus FETCH / WRITE
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS|FETCH_SIZE|WRITE_SIZE"
for gg in gate_up down; do
  PMC_GROUPS="$G" timeout -k 10 400 bash tools/pmc_sweep.sh r05_w4a4_$gg --cfg w4a4 --gg $gg --variants auto --iters 10 > $OUT/pmc_w4a4_bs8192_$gg.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_r05_w4a4_$gg/p*/
done
cat $OUT/pmc_w4a4_*.txt
