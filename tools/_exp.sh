set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp_b3tail.jsonl
for cfg in fp16 w8a8 mixed; do for gg in gate_up down; do
  timeout -k 10 120 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,18 --iters 40 --rounds 8 >> $O || exit $?
done; done
cat $O
