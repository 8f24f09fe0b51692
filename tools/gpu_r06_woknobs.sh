#!/bin/bash
# GPU box, round 6: planner knobs on the small-batch calls (lab copy of the product loop x_wo3_pch):
# tail chunk size, problem-aligned chunks off, plain round-robin chunks, band height
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-woknobs}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
V=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_wo3_pch'][0])")
for spec in "w4a16_w8a8 512" "w4a16_w8a8 128" "w4a16 512"; do
  set -- $spec
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $1 --gg $gg --bs $2 --variants $V,$V@MXMOE_GG_TAIL_CHUNK=8,$V@MXMOE_GG_TAIL_CHUNK=48,$V@MXMOE_GG_ALIGN=0,$V@MXMOE_GG_XCD_RR=1,$V@MXMOE_GG_BAND=1 --iters 60 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 6):
    g = rows[i:i + 6]
    base = g[0]["median_ms"]
    print(g[0]["cfg"], g[0]["bs"], g[0]["gg"], base, " ".join("%s %+.1f%%" % (r["spec"].split("@")[-1], 100 * (r["median_ms"] / base - 1)) for r in g[1:]))
PY
