#!/bin/bash
# GPU box, round 6: planner knobs (band height, n-group width, region rotation) re-checked under the
# whole-expert XCD packing, lab copy of the product kernel, bs 8192 layer calls, same process
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-knobs}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for cfg in fp16 w8a8 mixed; do
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --variants $VP,$VP@MXMOE_GG_BAND=2,$VP@MXMOE_GG_BAND=8,$VP@MXMOE_GG_NGROUP=2,$VP@MXMOE_GG_NGROUP=4,$VP@MXMOE_GG_REGION_ROT=1 --iters 60 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 6):
    g = rows[i:i + 6]
    base = g[0]["median_ms"]
    print(g[0]["cfg"], g[0]["gg"], base, " ".join("%s %+.1f%%" % (r["spec"].split("@")[-1], 100 * (r["median_ms"] / base - 1)) for r in g[1:]))
PY
