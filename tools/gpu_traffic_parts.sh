#!/bin/bash
# GPU box: PMC traffic of one layer call split into its routed experts and its shared expert, for
# the listed product variants.  usage: tools/gpu_traffic_parts.sh TAG "VARIANTS" [cfg] [gg]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VARS=$2; CFG=${3:-fp16}; GG=${4:-gate_up}
OUT=gpurun_out/parts_$TAG; mkdir -p $OUT; : > $OUT/summary.txt
export TMPDIR=/tmp
for v in $VARS; do
  for part in routed shared all; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      d=$OUT/${v}_${part}_${ctr}
      timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $d -o run -- \
        python3 tools/kbench.py --cfg $CFG --gg $GG --variants $v --only $part --iters 10 > $d.log 2>&1 || exit 1
    done
    python3 - $OUT $v $part >> $OUT/summary.txt <<'PY'
import csv, glob, sys
out, v, part = sys.argv[1:]
r = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = [float(x["Counter_Value"]) for f in glob.glob(f"{out}/{v}_{part}_{ctr}/**/*counter_collection.csv", recursive=True)
            for x in csv.DictReader(open(f)) if "gg_" in x.get("Kernel_Name", "") and x["Counter_Name"] == ctr]
    r[ctr] = sum(vals) / len(vals)
print(f"variant {v} {part}: fetch_x2 {2 * r['FETCH_SIZE'] * 1024 / 1e9:.3f} GB  write {r['WRITE_SIZE'] * 1024 / 1e9:.3f} GB")
PY
  done
done
find $OUT -name "*.csv" -delete
cat $OUT/summary.txt
