#!/bin/bash
# GPU box: FETCH_SIZE calibration on calls with a known byte count, and the gate_up call split into
# its routed and shared parts. One --pmc FETCH_SIZE kernel-trace pass per case.
set -o pipefail
TAG=${1:-calib}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, kbench args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$name -o run -- \
    python3 tools/kbench.py --variants auto --iters 10 "$@" > $OUT/$name.log 2>&1 || exit $?
  python3 - $OUT/$name "$name" <<'PY'
import csv, glob, sys
vals = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if "gg_" in r.get("Kernel_Name", "")]
print(sys.argv[2], "FETCH_SIZE x2 MB per dispatch:", round(2 * sum(vals) / len(vals) * 1024 / 1e6, 1), "n", len(vals))
PY
}
run dense_64x8192x4096 --cfg fp16 --dense 64,8192,4096
run dense_256x8192x4096 --cfg fp16 --dense 256,8192,4096
run fp16_gate_up_routed --cfg fp16 --gg gate_up --only routed
run fp16_gate_up_shared --cfg fp16 --gg gate_up --only shared
run w8a8_gate_up_routed --cfg w8a8 --gg gate_up --only routed
