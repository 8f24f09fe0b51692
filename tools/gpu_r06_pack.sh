#!/bin/bash
# GPU box, round 6: XCD packing placements (MXMOE_GG_XCD_PACK = 1 head / 2 tail / 3 head only for long
# region tiles) against the default placement on v2x, same process, many rounds; FETCH / WRITE
# counter passes of each placement on the fp16 and w8a8 calls; v4d stamp breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-pack}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
for cfg in fp16 w8a8; do
  for gg in gate_up down; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --variants 0,0@MXMOE_GG_XCD_PACK=1,0@MXMOE_GG_XCD_PACK=2,0@MXMOE_GG_XCD_PACK=3 --iters 80 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"], r["tflops"])
PY
timeout -k 10 200 python tools/stamps_v4.py --variant 2 --cfg w8a8 > $OUT/stamps_v4.jsonl 2>$OUT/stamps.err || { tail $OUT/stamps.err; exit 1; }
timeout -k 10 200 python tools/stamps_v4.py --variant 2 --cfg fp16 >> $OUT/stamps_v4.jsonl 2>>$OUT/stamps.err || exit 1
cat $OUT/stamps_v4.jsonl
for pk in 0 1 3; do
  for cfg in fp16 w8a8; do
    for gg in gate_up down; do
      PMC_GROUPS="FETCH_SIZE|WRITE_SIZE" timeout -k 10 200 bash tools/pmc_sweep.sh r06_pk${pk}_${cfg}_$gg --cfg $cfg --gg $gg --variants 0@MXMOE_GG_XCD_PACK=$pk --iters 6 --rounds 2 --settle-s 0.2 > $OUT/pmc_pk${pk}_${cfg}_$gg.txt 2>&1 || exit 1
      rm -rf gpurun_out/pmc_r06_pk${pk}_${cfg}_$gg/p*/
    done
  done
done
grep -H "SIZE" $OUT/pmc_pk*.txt
