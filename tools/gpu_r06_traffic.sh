#!/bin/bash
# GPU box, round 6: HBM counter bytes per bench step on this round's tree (FETCH_SIZE x2 + WRITE_SIZE,
# separate passes: tools/pmc_traffic.sh), every headline config incl. the small-batch scheme at bs 512,
# merged into one pmc_traffic.json tagged "round 6" (bench.py emits the tag as roofline.traffic_source)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PMC_ROUND="round 6"
mkdir -p gpurun_out/r06/traffic
PMC_OUT=gpurun_out/r06/traffic/b8192 timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 w4a4 mixed ds2_mixed > gpurun_out/r06/traffic_b8192.log 2>&1 || { tail -20 gpurun_out/r06/traffic_b8192.log; exit 1; }
PMC_OUT=gpurun_out/r06/traffic/b512 KB_ARGS="--bs 512" timeout -k 10 300 bash tools/pmc_traffic.sh w4a16_w8a8 > gpurun_out/r06/traffic_b512.log 2>&1 || { tail -20 gpurun_out/r06/traffic_b512.log; exit 1; }
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/r06/traffic/b8192/pmc_traffic.json"))
b = json.load(open("gpurun_out/r06/traffic/b512/pmc_traffic.json"))
a["w4a16_w8a8_bs512"] = b["w4a16_w8a8"]
a["_round"] = "round 6"
a["_method"] = a["_method"] + "; measured on the round-6 tree (XCD-packing planner): tools/gpu_r06_traffic.sh"
json.dump(a, open("gpurun_out/r06/traffic/pmc_traffic.json", "w"), indent=1)
for k, v in a.items():
    if isinstance(v, dict):
        print(k, round(v["hbm_bytes_per_step"] / 1e6, 1), "MB per step")
PY
find gpurun_out/r06/traffic -name "*.csv" -delete
