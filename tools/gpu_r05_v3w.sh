#!/bin/bash
# x_v3_256x256_w4_1wg (v3 at one wave per SIMD, 256 x 256 tiles) : parity on the GPU suite, then
# same-process kbench A/B against v3 (0) and v2x (1) on the int4 / mixed / w8a8 calls
set -o pipefail
OUT=gpurun_out/r05/${1:-v3w}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gg_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in w4a4 mixed ds2_mixed; do for gg in gate_up down; do
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 0,1,3 --iters 40 --rounds 8 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
done; done
timeout -k 10 200 python tools/kbench.py --cfg w4a4 --dense 8192,8192,8192 --variants 0,1,3 --iters 20 --rounds 4 >> $OUT/kbench.jsonl 2>>$OUT/kbench.err || exit 1
cat $OUT/kbench.jsonl
