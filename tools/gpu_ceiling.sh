#!/bin/bash
# GPU box: what the v2s schedule reaches with parts removed (timing ablations, WRONG RESULTS by
# design): 8 = v2s, 9 = no mainloop DMA, 10 = no epilogue stores, 11 = neither; int8 layer calls
# and dense 8192^3; then MFMA-busy / wait counters of variant 11 on dense 8192^3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_ceiling.jsonl
: > $OUT
for gg in gate_up down; do
  timeout -k 10 200 python tools/kbench.py --cfg w8a8 --gg $gg --variants 8,9,10,11 --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/kbench_ceiling.err || exit 1
done
timeout -k 10 200 python tools/kbench.py --cfg w8a8 --dense 8192,8192,8192 --variants 8,9,10,11 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_ceiling.err || exit 1
cut -c1-170 $OUT
PMC_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" timeout -k 10 300 bash tools/pmc_sweep.sh ceiling11 --cfg w8a8 --dense 8192,8192,8192 --variants 11 --iters 10 > gpurun_out/pmc_ceiling11.txt 2>&1 || exit 1
rm -rf gpurun_out/pmc_ceiling11/p*/
cat gpurun_out/pmc_ceiling11.txt
