#!/bin/bash
# GPU box, round 6: the small-batch fast loop with an L2 prefetch of B lines 8 stages ahead (lab
# x_wo3_pchpf) against x_wo3_pch and the round-5 loop (x_wo3): parity, then same-process kbench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-pf}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
timeout -k 10 300 python tools/wo_lab_parity.py --base x_wo3 --test x_wo3_pchpf > $OUT/parity.jsonl 2> $OUT/parity.err || { cat $OUT/parity.jsonl; tail -20 $OUT/parity.err; exit 1; }
cat $OUT/parity.jsonl
V=$(python -c "
from mxmoe_amd import _native as nat
n = {l.split()[1]: l.split()[0] for l in nat.list_variants()}
print(n['x_wo3'] + ',' + n['x_wo3_pch'] + ',' + n['x_wo3_pchpf'])")
for spec in "w4a16_w8a8 512" "w4a16_w8a8 128" "w4a16 512" "w4a16c 512"; do
  set -- $spec
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $1 --gg $gg --bs $2 --variants $V --iters 100 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for i in range(0, len(rows), 3):
    a, b, c = rows[i], rows[i + 1], rows[i + 2]
    print(a["cfg"], a["bs"], a["gg"], a["median_ms"], b["median_ms"], c["median_ms"],
          "pch %+.1f %%  pchpf %+.1f %%" % (100 * (b["median_ms"] / a["median_ms"] - 1), 100 * (c["median_ms"] / a["median_ms"] - 1)))
PY
