#!/bin/bash
# GPU box, round 6: the product placement (pack 4: whole experts, levelled shared pieces, head for long
# or 16-bit region tiles) against the round-5 placement (PACK=0) on the layer calls at bs 2048 / 4096 /
# 8192, gate_up and down, same process, lab copy of the product kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-plan4}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for bs in 2048 4096 8192; do
  for cfg in fp16 w8a8 mixed; do
    for gg in gate_up down; do
      timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants $VP@MXMOE_GG_XCD_PACK=0,$VP --iters 60 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
    done
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
base = {}
for r in rows:
    k = (r["cfg"], r["bs"], r["gg"])
    if "PACK=0" in r["spec"]:
        base[k] = r["median_ms"]
for r in rows:
    k = (r["cfg"], r["bs"], r["gg"])
    if "PACK=0" not in r["spec"]:
        print(*k, "pack0 %.4f  product %.4f  %+.1f %%" % (base[k], r["median_ms"], 100 * (r["median_ms"] / base[k] - 1)))
PY
