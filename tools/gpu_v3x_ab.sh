#!/bin/bash
# GPU box (fast lab): v3 256x128 2-WG/CU (7) vs v3x = + buffer-form DMA spread over the MFMAs (8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
OUT=gpurun_out/v3x_$1.jsonl; : > $OUT
timeout -k 10 300 python -u tools/lab_parity.py --variants 7,8 --cases fp16,w8a8,w4a4,mixed > gpurun_out/v3x_parity_$1.jsonl 2>gpurun_out/v3x_parity_$1.err || { tail -5 gpurun_out/v3x_parity_$1.err; grep '"ok": false' gpurun_out/v3x_parity_$1.jsonl; exit 1; }
echo parity ok
for cfg in w4a4 mixed w8a8; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 7,8$([ $cfg = w8a8 ] && echo ,0) --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/v3x_$1.err || exit 1
  done
done
timeout -k 10 200 python tools/kbench.py --cfg w4a4 --dense 8192,8192,8192 --variants 7,8 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/v3x_$1.err || exit 1
python - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["tflops"])
PY
