#!/bin/bash
# GPU box: lab-library mainloop experiments. Parity screen of the lab variants, then round-robin
# A/B (tools/kbench.py) on the layer-11 calls and dense 8192^3.
# usage: [STAMPS=i,j] [EXTRA="cfg:variants ..."] tools/gpu_lab_ab.sh TAG "VARIANTS" [cfgs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export MXMOE_GG_LIB=$PWD/mxmoe_amd/lib/libmxmoe_gg_lab.so
TAG=$1; VARS=$2; CFGS=${3:-"w8a8 fp16"}
mkdir -p gpurun_out
OUT=gpurun_out/lab_$TAG.jsonl
: > $OUT
PV=$(python -c "import sys; print(','.join(v for v in sys.argv[1].split(',') if v != '0'))" $VARS)
timeout -k 10 300 python -u tools/lab_parity.py --variants $PV > gpurun_out/lab_parity_$TAG.jsonl 2>gpurun_out/lab_parity_$TAG.err || { tail -5 gpurun_out/lab_parity_$TAG.err; grep '"ok": false' gpurun_out/lab_parity_$TAG.jsonl; exit 1; }
echo parity ok
for cfg in $CFGS; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $VARS --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/lab_$TAG.err || exit 1
  done
  timeout -k 10 200 python tools/kbench.py --cfg $cfg --dense 8192,8192,8192 --variants $VARS --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/lab_$TAG.err || exit 1
done
for cv in $EXTRA; do
  cfg=${cv%%:*}; vs=${cv#*:}
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants $vs --iters 40 --rounds 10 >> $OUT 2>>gpurun_out/lab_$TAG.err || exit 1
  done
done
cut -c1-150 $OUT
if [ -n "$STAMPS" ]; then
  timeout -k 10 300 python tools/stamps.py --variants $STAMPS --cfg w8a8 > gpurun_out/stamps_$TAG.jsonl 2>gpurun_out/stamps_$TAG.err || exit 1
  cat gpurun_out/stamps_$TAG.jsonl
fi
