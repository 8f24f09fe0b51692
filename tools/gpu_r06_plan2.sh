#!/bin/bash
# GPU box, round 6: XCD packing at other batch sizes (bs 4096 / 2048, where the shared expert still
# takes regions) and the head-placement alternative on the int calls: lab copy of the product kernel,
# round-5 placement (PACK=0) vs the product default vs always-head (PACK=1), same process
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-plan2}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for bs in 4096 2048; do
  for cfg in fp16 w8a8 mixed; do
    for gg in gate_up down; do
      timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants $VP@MXMOE_GG_XCD_PACK=0,$VP --iters 60 --rounds 15 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
    done
  done
done
for cfg in mixed ds2_mixed; do
  timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg gate_up --variants $VP@MXMOE_GG_XCD_PACK=0,$VP,$VP@MXMOE_GG_XCD_PACK=1 --iters 60 --rounds 15 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
