#!/bin/bash
# GPU box, round 6: (1) the headline measured five times in one box session (bench.py, headline only)
# to state the run-to-run spread beside the box-to-box one; (2) the product's AUTO kernels across
# batch sizes (qwen2_moe layer 11, gate_up + down, fp16 / w8a8 / w4a4 / mixed / w4a16_w8a8)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-sweep}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-scaling-sim --no-moe-layer --extras "" > $OUT/bench_$i.json 2>> $OUT/bench.err || exit 1
done
python3 - $OUT <<'PY'
import json, sys, glob
vals = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json"))]
print("headline runs:", [round(v["value"], 1) for v in vals], "frac", [v["roofline"]["frac"] for v in vals])
PY
for cfg in fp16 w8a8 w4a4 mixed w4a16_w8a8; do
  for bs in 128 512 2048 8192 16384; do
    for gg in gate_up down; do
      timeout -k 10 300 python tools/kbench.py --cfg $cfg --gg $gg --bs $bs --variants auto --iters 40 --rounds 4 --settle-s 0.3 >> $OUT/sweep.jsonl 2>>$OUT/sweep.err || exit 1
    done
  done
done
python3 - $OUT/sweep.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for r in rows:
    print(r["cfg"], r["bs"], r["gg"], r["variant"], r["median_ms"], r["tflops"], r["gbs"])
PY
