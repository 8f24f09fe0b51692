#!/bin/bash
# GPU box, round 6: the planner's live-row cost for row-skipping weight-only tiles (full 64-row tiles
# sort first) against the flat 64-row cost (MXMOE_GG_WO_ROWCOST=0), lab copy of the product loop;
# then the tile timeline of the bs 512 gate_up call with it
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-rowcost}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
V=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_wo3_pch'][0])")
for spec in "w4a16_w8a8 512" "w4a16_w8a8 128" "w4a16 512" "w4a16c 512" "w4a16_w8a8 1024" "w4a16 2048"; do
  set -- $spec
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $1 --gg $gg --bs $2 --variants $V@MXMOE_GG_WO_ROWCOST=0,$V,$V@MXMOE_GG_WO_ROWCOST=2 --iters 100 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 3):
    a, b, c = rows[i], rows[i + 1], rows[i + 2]
    print(a["cfg"], a["bs"], a["gg"], a["median_ms"], b["median_ms"], c["median_ms"], "order %+.1f %%  order+sim %+.1f %%" % (100 * (b["median_ms"] / a["median_ms"] - 1), 100 * (c["median_ms"] / a["median_ms"] - 1)))
PY
timeout -k 10 120 python tools/tile_trace.py --cfg w4a16_w8a8 --gg gate_up --bs 512 --variant-name abl_wo3_pch_trace --dump $OUT/trace_gate_up.npy >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit 1
