#!/bin/bash
# GPU box: does a non-power-of-two row stride (A / B rows padded by 128 / 256 B) change L2 reuse?
# kbench A/B + PMC FETCH_SIZE of the padded inputs.
set -o pipefail
TAG=${1:-pad}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
# padded rows give the same C bit for bit (fp16, w8a8 layer at bs=1024)
timeout -k 10 120 python - <<'PY' || exit 1
import sys, torch
sys.path.insert(0, "tools")
from kbench import padded
from mxmoe_amd.groupgemm import GroupGemm
from mxmoe_amd.harness import build_layer_inputs
from mxmoe_amd.workload import load_workload, qwen2_layer11_workload
for kw in ({}, dict(qstr="w8a8_g-1_sym")):
    for gg in ("gate_up", "down"):
        base = build_layer_inputs(load_workload(qwen2_layer11_workload(1024, **kw))["layer-11"][gg])
        pad = padded(base, 128)
        for p in pad.problems:
            p.C = torch.full_like(p.C, float("nan"))
        GroupGemm(base.problems).launch(); GroupGemm(pad.problems).launch(); torch.cuda.synchronize()
        for a, b in zip(base.problems, pad.problems):
            if a.M:
                assert torch.equal(a.C.view(torch.int16), b.C.view(torch.int16)), (kw, gg, a.M, a.N, a.K)
print("padded-row parity ok")
PY
for cg in "fp16 gate_up" "fp16 down" "w8a8 gate_up" "w8a8 down"; do
  set -- $cg
  timeout -k 10 150 python tools/kbench.py --cfg $1 --gg $2 --variants auto --pads 0,128,256 --iters 40 --rounds 8 >> gpurun_out/$TAG/kbench_pad_ab.jsonl || exit 1
done
cat gpurun_out/$TAG/kbench_pad_ab.jsonl
KB_ARGS="--pads 128" PMC_OUT=gpurun_out/$TAG/pmc_pad128 timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 > gpurun_out/$TAG/pmc_pad128.log 2>&1 || { tail -20 gpurun_out/$TAG/pmc_pad128.log; exit 1; }
grep -A3 '"gate_up"\|"down"' gpurun_out/$TAG/pmc_pad128/pmc_traffic.json | grep -v write
