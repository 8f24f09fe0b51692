#!/bin/bash
# GPU box: bench.py at the driver's --warmup 5 with / without the plan-then-materialise order (x2 each)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04/warm
mkdir -p $OUT
for i in 1 2; do
  for m in --materialise-after-plan --no-materialise-after-plan; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras "" --no-scaling-sim --no-cpu-baseline $m > $OUT/b_${i}_$m.json 2> $OUT/b_${i}_$m.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/b_${i}_$m.json')); print('$m', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  done
done
