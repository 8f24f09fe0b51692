#!/bin/bash
# GPU box, round 6: long-pole priority in the small-batch loop (lab x_wo3_pch_prio) against x_wo3_pch:
# parity, same-process kbench on the bs 512 / 128 calls, and the down call's tile timeline with it
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-prio}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
timeout -k 10 300 python tools/wo_lab_parity.py --base x_wo3 --test x_wo3_pch_prio > $OUT/parity.jsonl 2> $OUT/parity.err || { cat $OUT/parity.jsonl; tail -20 $OUT/parity.err; exit 1; }
V=$(python -c "
from mxmoe_amd import _native as nat
n = {l.split()[1]: l.split()[0] for l in nat.list_variants()}
print(n['x_wo3_pch'] + ',' + n['x_wo3_pch_prio'])")
for spec in "w4a16_w8a8 512" "w4a16_w8a8 128" "w4a16 512" "w4a16c 512" "w4a16_w8a8 1024"; do
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
for gg in gate_up down; do
  timeout -k 10 120 python tools/tile_trace.py --cfg w4a16_w8a8 --gg $gg --bs 512 --variant-name abl_wo3_pch_prio_trace --dump $OUT/trace_$gg.npy >> $OUT/trace.jsonl 2>> $OUT/trace.err || exit 1
done
