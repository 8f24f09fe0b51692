#!/bin/bash
# GEMM kernels of two builds, alternating processes (AUTO variant): tools/gpu_r05_kab.sh TAG LIB_A LIB_B [cfgs]
set -o pipefail
TAG=$1; LA=$2; LB=$3; CFGS=${4:-fp16 w8a8 mixed}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
for rep in 1 2; do for lib in $LA $LB; do for cfg in $CFGS; do for gg in gate_up down; do
  MXMOE_GG_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants auto --iters 40 --rounds 4 \
    | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done; done; done; done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(r["cfg"], r["gg"], r["lib"].split("/")[-1])].append(r["median_ms"])
for k in sorted(d): print(k, d[k])
PY
