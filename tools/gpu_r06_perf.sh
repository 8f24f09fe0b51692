#!/bin/bash
# GPU box, round 6: the performance table's w8a8 / w4a4 / fp16 rows re-measured on today's AUTO
# kernels (tools/perf_table.py into a copy of the committed table) and the cost model checked against
# the layer-11 calls with the committed and the re-measured table (tools/perf_table_check.py); the
# small-batch interleave knob (MXMOE_GG_MIX) on wo3 (fast lab library)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-perf}
mkdir -p $OUT
timeout -k 10 200 python tools/perf_table_check.py --bs 8192,4096 > $OUT/check_committed.json 2> $OUT/check.err || { tail $OUT/check.err; exit 1; }
cat $OUT/check_committed.json
cp mxmoe_amd/workloads/performance_table_mi355x.json $OUT/performance_table_mi355x.json
timeout -k 10 600 python tools/perf_table.py --qcfgs w4a4_g-1_sym,w8a8_g-1_sym,fp16 --merge --out $OUT/performance_table_mi355x.json > $OUT/sweep.log 2>&1 || { tail $OUT/sweep.log; exit 1; }
timeout -k 10 200 python tools/perf_table_check.py --bs 8192,4096 --table $OUT/performance_table_mi355x.json > $OUT/check_remeasured.json 2>> $OUT/check.err || exit 1
cat $OUT/check_remeasured.json
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VW=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_wo3'][0])")
for cfg in w4a16_w8a8 w4a16; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --bs 512 --variants $VW,$VW@MXMOE_GG_MIX=1 --iters 80 --rounds 20 >> $OUT/kbench_mix.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench_mix.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
