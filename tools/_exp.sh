set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_b3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_b3.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_b3.log
O=gpurun_out/exp_b3c.jsonl
for cfg in fp16 w8a8 mixed; do for gg in gate_up down; do
  timeout -k 10 120 python tools/kbench.py --cfg $cfg --gg $gg --variants 8,17,auto --iters 40 --rounds 8 >> $O || exit $?
done; done
cat $O
