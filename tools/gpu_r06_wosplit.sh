#!/bin/bash
# GPU box, round 6: the small-batch wo3 calls fill ~1.3 rounds of the 768 workgroup
# slots; K-sliced tails / more split-K retried under the write-through split-K hand-off (round 4), which
# the round-3 measurements of the same knobs predate. Same process, lab copy of wo3.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-wosplit}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
W=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_wo3'][0])")
for cfg in w4a16_w8a8 w4a16; do
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --bs 512 --variants $W,$W@MXMOE_GG_TAIL_SPLIT=2,$W@MXMOE_GG_SPLIT_RATIO_MUL=1.5,$W@MXMOE_GG_SPLITK_ALL=2,$W@MXMOE_GG_SPLIT_RATIO_MUL=0.5 --iters 100 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tiles"], r["grid"])
PY
