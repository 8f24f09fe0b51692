#!/bin/bash
# GPU box, round 4: split-K hand-off parity (the suites that run split-K), wo3 lab A/B, and a
# re-measured w4a4 row of the performance table. usage: tools/gpu_r04_mix.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-mix}
OUT=gpurun_out/r04/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gg_gpu.py tests/test_weightonly_gpu.py tests/test_fp8_bf16_gpu.py tests/test_moe.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_r04_wo.sh $TAG 9,10 9,10,9@MXMOE_GG_SPLIT_RATIO_MUL=1.3,9@MXMOE_GG_SPLITK_ALL=2,9@MXMOE_GG_REGION=1,9@MXMOE_GG_REGION=0,9@MXMOE_GG_LOWFILL_LPT=1 "w4a16_w8a8 w4a16" "512 128" > $OUT/wo.log 2>&1 || { tail -20 $OUT/wo.log; exit 1; }
cp mxmoe_amd/workloads/performance_table_mi355x.json $OUT/performance_table_mi355x.json
timeout -k 10 900 python -u tools/perf_table.py --qcfgs w4a4_g-1_sym --merge --out $OUT/performance_table_mi355x.json > $OUT/perf_table.log 2>&1 || { tail -20 $OUT/perf_table.log; exit 1; }
echo perf table ok
