#!/bin/bash
# GPU box, round 6: the -m gpu suite, smoke(), bench.py (JSON line) + rocprofv3 kernel stats of the
# same command, and counter passes (MFMA busy, wait split, L2 hit, LDS conflicts) of the AUTO kernels
# on the bs=8192 gate_up calls of fp16 / w8a8 / w4a4 / mixed.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-check}
OUT=gpurun_out/r06/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 bench.py --no-cpu-baseline --no-scaling-sim --extras "" > $OUT/bench_prof.json 2> $OUT/prof.err || exit 1
rm -f $OUT/prof/run_kernel_trace.csv
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
for cfg in ${PMC_CFGS:-w4a4 mixed w8a8 fp16}; do
  PMC_GROUPS="$G" timeout -k 10 300 bash tools/pmc_sweep.sh r06_${TAG}_$cfg --cfg $cfg --gg gate_up --variants auto --iters 10 > $OUT/pmc_${cfg}_bs8192_gate_up.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_r06_${TAG}_$cfg/p*/
done
cat $OUT/pmc_*.txt
