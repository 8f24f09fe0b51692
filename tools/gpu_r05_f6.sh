#!/bin/bash
# fp6-image w4a4 path: parity tests, then int4 vs fp6 timing on the w4a4 layer calls
set -o pipefail
OUT=gpurun_out/f6/${1:-run1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_f6.py tests/test_abi.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
MXMOE_GG_LIB=mxmoe_amd/lib/libmxmoe_gg_lab.so timeout -k 10 400 python -u tools/f6_bench.py --out $OUT/bench.json --f6-variants "${F6V:-}" > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
cat $OUT/bench.log
