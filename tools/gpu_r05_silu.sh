#!/bin/bash
# fused SiLU epilogue: parity (new tests + the GEMM / MoE / golden GPU suites), MoE layer step
# fused vs unfused, and the GEMM kernels against the previous build (no regression of the plain
# epilogue path): tools/gpu_r05_silu.sh TAG BASE_LIB
set -o pipefail
TAG=${1:-silu1}; BASE=${2:-mxmoe_amd/lib/libmxmoe_gg_base.so}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_silu_epi.py tests/test_moe.py tests/test_gg_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/moe_layer_bench.py > $OUT/moe_layer.jsonl 2> $OUT/moe_layer.err || { tail -20 $OUT/moe_layer.err; exit 1; }
cat $OUT/moe_layer.jsonl
for rep in 1 2; do for lib in $BASE mxmoe_amd/lib/libmxmoe_gg.so; do for cfg in fp16 w8a8 mixed; do for gg in gate_up down; do
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
