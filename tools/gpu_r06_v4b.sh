#!/bin/bash
# GPU box, round 6: v4d (+ LDS scale stash) parity + same-process A/B vs v2x, with and without the
# XCD packing knob, more rounds; counter passes of both kernels on dense int8 8192^3
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-v4b}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
timeout -k 10 300 python tools/lab_parity.py --variants 1 --cases fp16,w8a8 > $OUT/parity.jsonl 2> $OUT/parity.err || { tail -5 $OUT/parity.jsonl; tail -20 $OUT/parity.err; exit 1; }
grep -c '"ok": true' $OUT/parity.jsonl
for cfg in w8a8 fp16; do
  timeout -k 10 240 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 0,1 --iters 30 --rounds 10 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --variants 0,1,0@MXMOE_GG_XCD_PACK=1,1@MXMOE_GG_XCD_PACK=1 --iters 60 --rounds 15 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
G="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES|SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE|SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS|TCC_HIT_sum TCC_MISS_sum"
for v in 0 1; do
  PMC_GROUPS="$G" timeout -k 10 300 bash tools/pmc_sweep.sh r06_dense_v$v --cfg w8a8 --dense 8192,8192,8192 --variants $v --iters 10 --rounds 2 --settle-s 0.5 > $OUT/pmc_dense_w8a8_v$v.txt 2>&1 || exit 1
  rm -rf gpurun_out/pmc_r06_dense_v$v/p*/
done
cat $OUT/pmc_dense_*.txt
