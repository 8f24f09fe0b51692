#!/bin/bash
# GPU box, round 6: where the shared expert's pieces go at bs 2048 / 4096 (gate_up calls): round-5
# placement (PACK=0), always head (1), head only for long region tiles (3), product default, same process
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-plan3}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for bs in 2048 4096; do
  for cfg in fp16 w8a8 mixed; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg gate_up --bs $bs --variants $VP@MXMOE_GG_XCD_PACK=0,$VP@MXMOE_GG_XCD_PACK=1,$VP@MXMOE_GG_XCD_PACK=3,$VP --iters 80 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
