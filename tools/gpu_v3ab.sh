set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=gpurun_out/kbench_v3ab.jsonl
: > $OUT
for cfg in w8a8 fp16 w4a4; do
  for gg in gate_up down; do
    timeout -k 10 200 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,7,4 --iters 20 --rounds 5 >> $OUT 2>>gpurun_out/kbench_v3ab.err || exit 1
  done
done
cat $OUT
