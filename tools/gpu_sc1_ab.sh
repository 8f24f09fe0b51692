#!/bin/bash
# GPU box: C stores with sc1 (drop the line from L2) vs plain — parity with the sc1 library, kbench
# in alternating processes (each library is one process), FETCH/WRITE traffic of the sc1 library.
set -o pipefail
TAG=${1:-sc1}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
SC1=$GRAFT_REPO_ROOT/mxmoe_amd/lib/libmxmoe_gg_sc1.so
MXMOE_GG_LIB=$SC1 timeout -k 10 300 python -u -m pytest tests/test_gg_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_sc1.log 2>&1 || { tail -30 $OUT/pytest_sc1.log; exit 1; }
tail -1 $OUT/pytest_sc1.log
for rep in 1 2; do
  for lib in plain sc1; do
    for cg in "fp16 gate_up" "fp16 down" "w8a8 gate_up" "w8a8 down"; do
      set -- $cg
      if [ $lib = sc1 ]; then export MXMOE_GG_LIB=$SC1; else unset MXMOE_GG_LIB; fi
      timeout -k 10 120 python tools/kbench.py --cfg $1 --gg $2 --variants auto --iters 40 --rounds 4 | sed "s/^{/{\"lib\": \"$lib\", \"rep\": $rep, /" >> $OUT/kbench.jsonl || exit 1
    done
  done
done
unset MXMOE_GG_LIB
MXMOE_GG_LIB=$SC1 PMC_OUT=$OUT/pmc_sc1 timeout -k 10 900 bash tools/pmc_traffic.sh fp16 w8a8 > $OUT/pmc_sc1.log 2>&1 || { tail -20 $OUT/pmc_sc1.log; exit 1; }
find $OUT/pmc_sc1 -name "*.csv" -delete
grep hbm_bytes_per_step $OUT/pmc_sc1/pmc_traffic.json
