#!/bin/bash
# GPU box, round 5: the MoE plumbing kernels (tools/moe_bench.py) — timing, then one --pmc group per
# run (kernel-trace only) for act_quant_kernel (quant_act / silu_mul_quant) and combine_kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05/${1:-moepmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/moe_bench.py --iters 30 > $OUT/moe_bench.jsonl 2> $OUT/moe_bench.err || { tail -20 $OUT/moe_bench.err; exit 1; }
cat $OUT/moe_bench.jsonl
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE TA_BUSY_avr" "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/moe_bench.py --iters 5 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:70]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "act_quant" not in k and "combine" not in k and "route" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
rm -rf $OUT/p*/
