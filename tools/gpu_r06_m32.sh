#!/bin/bash
# GPU box, round 6: timing of the small-batch loop with its MFMAs issued as 32x32x16 (lab ablation
# abl_wo3_pch_m32, WRONG RESULTS by design) against the product loop's copy (x_wo3_pch), same process
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-m32}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
V=$(python -c "
from mxmoe_amd import _native as nat
n = {l.split()[1]: l.split()[0] for l in nat.list_variants()}
print(n['x_wo3_pch'] + ',' + n['abl_wo3_pch_m32'])")
for spec in "w4a16_w8a8 512" "w4a16_w8a8 128" "w4a16c 512" "w4a16 512"; do
  set -- $spec
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $1 --gg $gg --bs $2 --variants $V --iters 100 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 2):
    a, b = rows[i], rows[i + 1]
    print(a["cfg"], a["bs"], a["gg"], a["median_ms"], b["median_ms"], "%+.1f %%" % (100 * (b["median_ms"] / a["median_ms"] - 1)))
PY
