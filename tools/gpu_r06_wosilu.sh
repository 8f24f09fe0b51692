#!/bin/bash
# GPU box, round 6 (VERDICT r05 missing item 5): the small-batch kernel's fused SiLU epilogue — the
# SiLU GPU tests, then the bs 512 MoE layer unfused / fused (wo3 epilogue) / interleaved (plain wo3
# epilogue + the interleaved-input SiLU pass), and the same at bs 8192 for reference
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06/${1:-wosilu}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_silu_epi.py tests/test_abi.py tests/test_moe.py tests/test_weightonly_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python - > $OUT/moe_layer.jsonl 2> $OUT/moe_layer.err <<'PY' || { tail -20 $OUT/moe_layer.err; exit 1; }
import json
from mxmoe_amd.moe import qwen2_layer_bench
for scheme, bs in (("w4a16_w8a8", 512), ("w4a16_w8a8", 128), ("lp1", 512), ("lp1", 128), ("lp1", 2048)):
    r = qwen2_layer_bench(rounds=3, iters=30, bs=bs, interleaved=True, scheme=scheme)
    print(json.dumps({"scheme": scheme, "bs": bs, **r}), flush=True)
PY
cat $OUT/moe_layer.jsonl
