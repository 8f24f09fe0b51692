#!/bin/bash
# GPU box, round 6: the int gate_up calls at bs 4096, where the product placement read 2-3 % slower than
# the round-5 one: repeat A/B (two processes) and the FETCH / WRITE counter bytes of each placement
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-b4096}
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
VP=$(python -c "
from mxmoe_amd import _native as nat
print([l.split()[0] for l in nat.list_variants() if l.split()[1] == 'x_v2x_product'][0])")
for rep in 1 2; do
  for cfg in w8a8 mixed; do
    timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg gate_up --bs 4096 --variants $VP@MXMOE_GG_XCD_PACK=0,$VP,$VP@MXMOE_GG_XCD_PACK=1 --iters 60 --rounds 20 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["cfg"], r["bs"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"])
PY
for pk in 0 4; do
  for cfg in w8a8 mixed; do
    PMC_GROUPS="FETCH_SIZE|WRITE_SIZE" timeout -k 10 200 bash tools/pmc_sweep.sh r06_b4096_pk${pk}_${cfg} --cfg $cfg --gg gate_up --bs 4096 --variants $VP@MXMOE_GG_XCD_PACK=$pk --iters 6 --rounds 2 --settle-s 0.2 > $OUT/pmc_pk${pk}_${cfg}.txt 2>&1 || exit 1
    rm -rf gpurun_out/pmc_r06_b4096_pk${pk}_${cfg}/p*/
  done
done
grep -H "SIZE" $OUT/pmc_pk*.txt
