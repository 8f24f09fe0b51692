#!/bin/bash
# GPU box: counters of wo3 (9) vs v2x (8) on the small-batch weight-only / mixed calls
# (w4a16 g128 asym at bs 512, gate_up), and the HBM traffic of the AUTO variant per step
# (w4a16 bs 512 -> wo3; tools/pmc_traffic.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/wo3_evidence; mkdir -p $OUT
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum"
for v in 8 9; do
  for gg in gate_up down; do
    PMC_GROUPS="$G" timeout -k 10 400 bash tools/pmc_sweep.sh wo3_${v}_$gg --cfg w4a16 --bs 512 --gg $gg --variants $v --iters 10 > $OUT/pmc_w4a16_bs512_${gg}_v$v.txt 2>&1 || exit 1
    rm -rf gpurun_out/pmc_wo3_${v}_$gg/p*/
  done
done
cat $OUT/pmc_*.txt
PMC_OUT=gpurun_out/wo3_evidence/traffic KB_ARGS="--bs 512" timeout -k 10 900 bash tools/pmc_traffic.sh w4a16 || exit 1
cat gpurun_out/wo3_evidence/traffic/pmc_traffic.json
