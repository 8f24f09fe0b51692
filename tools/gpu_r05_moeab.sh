#!/bin/bash
# GPU box, round 5: MoE plumbing parity (tests/test_moe.py) on the new build, then tools/moe_bench.py
# on two builds in alternating processes: usage tools/gpu_r05_moeab.sh TAG LIB_A LIB_B [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; LA=$2; LB=$3; REPS=${4:-3}
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_moe.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in $(seq 1 $REPS); do
  for lib in $LA $LB; do
    MXMOE_GG_LIB=$PWD/$lib timeout -k 10 200 python tools/moe_bench.py --iters 50 \
      | sed "s|^{|{\"lib\": \"$lib\", \"rep\": $rep, |" >> $OUT/moe_bench.jsonl 2>>$OUT/moe_bench.err || exit 1
  done
done
python3 - $OUT/moe_bench.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    d[(r["kernel"], r["lib"])].append(r["median_us"])
for k in sorted(d):
    print(k, d[k])
PY
