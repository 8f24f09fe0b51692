#!/bin/bash
# GPU box, round 4: counter passes (MFMA busy, issue / wait split, L2 hit) of the product AUTO
# kernels: wo3 on the bs 512 w4a16 + w8a8 calls, v2x on the w8a8 / fp16 bs 8192 gate_up calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04/busy; mkdir -p $OUT
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum"
for spec in "w4a16_w8a8 512 gate_up" "w4a16_w8a8 512 down" "w8a8 8192 gate_up" "fp16 8192 gate_up"; do
  set -- $spec
  PMC_GROUPS="$G" timeout -k 10 400 bash tools/pmc_sweep.sh r04_$1_$2_$3 --cfg $1 --bs $2 --gg $3 --variants auto --iters 10 > $OUT/pmc_$1_bs$2_$3.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_r04_$1_$2_$3/p*/
done
cat $OUT/pmc_*.txt
