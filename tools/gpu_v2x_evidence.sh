#!/bin/bash
# GPU box: dense 8192^3 and layer-11 timing of v2x (8) vs v2s (6), then MFMA-busy / wait / clock /
# L2 counters of v2x on dense 8192^3 (int8, fp16) and the w8a8 gate_up call.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/v2x_evidence; mkdir -p $OUT; : > $OUT/kbench.jsonl
for cfg in w8a8 fp16; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 6,8 --iters 20 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done
cut -c1-160 $OUT/kbench.jsonl
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|TCC_HIT_sum TCC_MISS_sum"
for c in "dense_w8a8:--cfg w8a8 --dense 8192,8192,8192" "dense_fp16:--cfg fp16 --dense 8192,8192,8192" "w8a8_gate_up:--cfg w8a8 --gg gate_up" "fp16_gate_up:--cfg fp16 --gg gate_up"; do
  tag=${c%%:*}; args=${c#*:}
  PMC_GROUPS="$G" timeout -k 10 400 bash tools/pmc_sweep.sh v2x_$tag $args --variants 8 --iters 10 > $OUT/pmc_$tag.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_v2x_$tag/p*/
done
cat $OUT/pmc_*.txt
