#!/bin/bash
# GPU box, round 6: band height 8 vs the default 4 on the fp16 / w8a8 bs 8192 calls, repeated in three
# processes (lab copy of the product kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-band}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for rep in 1 2 3; do
  for cfg in fp16 w8a8; do
    for gg in gate_up down; do
      timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --variants $VP,$VP@MXMOE_GG_BAND=8 --iters 60 --rounds 30 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
    done
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 2):
    a, b = rows[i], rows[i + 1]
    print(a["cfg"], a["gg"], a["median_ms"], b["median_ms"], "%+.1f %%" % (100 * (b["median_ms"] / a["median_ms"] - 1)))
PY
