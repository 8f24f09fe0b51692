#!/bin/bash
# GPU box, round 6: counters of the small-batch gate_up call (w4a16 + w8a8, bs 512) on the round-5
# loop (lab x_wo3) and the product loop (x_wo3_pch): instruction mix, issue activity, MFMA busy
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-wopmc}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
V=$(python -c "
from mxmoe_amd import _native as nat
n = {l.split()[1]: l.split()[0] for l in nat.list_variants()}
print(n['x_wo3'] + ',' + n['x_wo3_pch'])")
for gg in gate_up down; do
  PMC_GROUPS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
    timeout -k 10 400 bash tools/pmc_sweep.sh r06_wopmc_$gg --cfg w4a16_w8a8 --gg $gg --bs 512 --variants $V --iters 10 --rounds 2 --settle-s 0.2 > $OUT/pmc_$gg.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_r06_wopmc_$gg/p*/
done
cat $OUT/pmc_*.txt
