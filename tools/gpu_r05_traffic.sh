#!/bin/bash
# GPU box, round 5: placement knobs of the lab planner — same-process round-robin timing (kbench)
# and FETCH_SIZE / WRITE_SIZE passes per knob setting (separate --pmc runs, kernel trace only).
# usage: tools/gpu_r05_traffic.sh TAG VARIANT "cfgs" "knob specs (ENV=VAL, '-' = default)"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; V=$2; CFGS=$3; KNOBS=$4
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
export TMPDIR=/tmp
SPECS=""
for k in $KNOBS; do if [ "$k" = "-" ]; then SPECS="$SPECS,$V"; else SPECS="$SPECS,$V@$k"; fi; done
SPECS=${SPECS#,}
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 240 python tools/kbench.py --cfg $cfg --gg $gg --variants $SPECS --iters 40 --rounds 10 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
  done
done
i=0
for k in $KNOBS; do
  i=$((i+1))
  for cfg in $CFGS; do
    for gg in gate_up down; do
      for ctr in FETCH_SIZE WRITE_SIZE; do
        if [ "$k" = "-" ]; then ENVK=""; else ENVK="$k"; fi
        ( [ -n "$ENVK" ] && export "$ENVK"; timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/k${i}_${cfg}_${gg}_${ctr} -o run -- \
          python3 tools/kbench.py --cfg $cfg --gg $gg --variants $V --iters 10 --rounds 2 --settle-s 0.2 > $OUT/k${i}_${cfg}_${gg}_${ctr}.log 2>&1 ) || exit 1
      done
    done
  done
done
python3 - $OUT "$CFGS" "$KNOBS" <<'PY'
import csv, glob, json, sys
out, cfgs, knobs = sys.argv[1], sys.argv[2].split(), sys.argv[3].split()
res = {}
for i, k in enumerate(knobs, 1):
    for cfg in cfgs:
        tot = 0.0
        for gg in ("gate_up", "down"):
            v = {}
            for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
                vals = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/k{i}_{cfg}_{gg}_{ctr}/**/*counter_collection.csv", recursive=True)
                        for r in csv.DictReader(open(f)) if "gg_" in r.get("Kernel_Name", "") and r["Counter_Name"] == ctr]
                v[ctr] = sum(vals) / max(1, len(vals))
            b = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
            res[f"{k}|{cfg}|{gg}"] = round(b / 1e6, 1)
            tot += b
        res[f"{k}|{cfg}|step"] = round(tot / 1e6, 1)
json.dump(res, open(f"{out}/traffic.json", "w"), indent=1)
for k, v in res.items(): print(k, v, "MB")
for l in open(f"{out}/kbench.jsonl"):
    r = json.loads(l); print(r["cfg"], r["gg"], r["spec"], r["median_ms"], r["spread_ms"])
PY
