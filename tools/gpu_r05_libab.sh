#!/bin/bash
# GPU box, round 5: parity of the int paths on the new build, then an A/B of two builds of the same
# variant in alternating processes: usage tools/gpu_r05_libab.sh TAG LIB_A LIB_B VARIANT "cfgs" "bss" [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; LA=$2; LB=$3; V=$4; CFGS=$5; BSS=$6; KEXPR=${7:-}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for rep in 1 2; do
  for lib in $LA $LB; do
    for bs in $BSS; do
      for cfg in $CFGS; do
        for gg in gate_up down; do
          MXMOE_GG_LIB=$PWD/$lib timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants $V --iters 40 --rounds 8 \
            | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
        done
      done
    done
  done
done
python3 - $OUT/kbench.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
d = collections.defaultdict(list)
for r in rows:
    d[(r["cfg"], r["bs"], r["gg"], r["lib"])].append(r["median_ms"])
for k in sorted(d):
    print(k, [round(x, 4) for x in d[k]])
PY
