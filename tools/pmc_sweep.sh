#!/bin/bash
# Counter passes (one --pmc group per run, kernel-trace only) for tools/kbench.py args.
# usage: bash tools/pmc_sweep.sh <tag> <kbench args...>
set -o pipefail
TAG=$1; shift
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd $REPO
export TMPDIR=/tmp
i=0
PMC_LIST=${PMC_GROUPS:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA|SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY|SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE|FETCH_SIZE|TCC_HIT_sum TCC_MISS_sum|WRITE_SIZE TA_BUSY_avr TCP_TCC_READ_REQ_sum"}
IFS='|' read -ra GRPS <<< "$PMC_LIST"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/kbench.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "gg_" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
