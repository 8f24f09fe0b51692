#!/bin/bash
# MoE layer step (tools/moe_layer_bench.py) on two builds, alternating processes, after the SiLU /
# MoE parity tests: tools/gpu_r05_siluab.sh TAG LIB_A LIB_B [reps]
set -o pipefail
TAG=$1; LA=$2; LB=$3; REPS=${4:-2}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_silu_epi.py tests/test_moe.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in $(seq 1 $REPS); do for lib in $LA $LB; do
  MXMOE_GG_LIB=$PWD/$lib timeout -k 10 300 python tools/moe_layer_bench.py --rounds 3 \
    | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $OUT/moe_layer.jsonl 2>>$OUT/moe_layer.err || exit 1
done; done
python3 - $OUT/moe_layer.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["lib"].split("/")[-1], r["rep"], "unfused", r["unfused"]["step"], r["unfused"]["act_quant"], "fused", r["fused"]["step"], r["fused"]["gate_up"], r["fused"]["act_quant"], r["bit_identical"])
PY
