#!/bin/bash
# GPU box, round 4: the new boundary / share_fused tests, then the store-path probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ref_harness.py tests/test_moe.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -30 $OUT/pytest_new.log; exit 1; }
tail -4 $OUT/pytest_new.log
timeout -k 10 120 tools/bin/store_probe > $OUT/store_probe.jsonl 2> $OUT/store_probe.err || { cat $OUT/store_probe.err; exit 1; }
cat $OUT/store_probe.jsonl
