#!/bin/bash
# GPU box, round 6: v4d (gg_v4.h, one wave per SIMD) parity screen + dense 8192^3 and layer-call A/B
# against v2x in one process (fast lab library), and the XCD packing planner knob (MXMOE_GG_XCD_PACK)
# on v2x's layer calls.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-v4a}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
timeout -k 10 300 python tools/lab_parity.py --variants 1 --cases fp16,w8a8 > $OUT/parity.jsonl 2> $OUT/parity.err || { tail -5 $OUT/parity.jsonl; tail -20 $OUT/parity.err; exit 1; }
tail -3 $OUT/parity.jsonl
for cfg in w8a8 fp16; do
  timeout -k 10 240 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants 0,1 --iters 20 --rounds 5 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  for gg in gate_up down; do
    timeout -k 10 240 python tools/kbench.py --cfg $cfg --gg $gg --variants 0,1,0@MXMOE_GG_XCD_PACK=1 --iters 40 --rounds 10 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
