#!/bin/bash
# GPU box, round 6: the XCD-packing planner (product default) — full-size sampled parity and golden
# vectors on the product library, then same-process A/B of the lab library's product kernel with the
# round-5 placement (MXMOE_GG_XCD_PACK=0) against the new default on every bs 8192 bench config, and
# the perf-table / small-batch screen (gpu_r06_perf.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-plan}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_golden_gpu.py tests/test_planner.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
VP=$(MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
echo "x_v2x_product = $VP"
for cfg in fp16 w8a8 mixed ds2_mixed bf16 w4a16; do
  for gg in gate_up down; do
    MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg \
      --variants $VP@MXMOE_GG_XCD_PACK=0,$VP --iters 80 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
