# GPU box: the N > 1 code path rehearsed on one GPU (2 ranks, gloo), its GPU test, then the N = 1 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_cli_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1 || { tail -40 gpurun_out/pytest_dist.log; exit 1; }
tail -3 gpurun_out/pytest_dist.log
MXMOE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --extras "" \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
cat gpurun_out/bench_n2_gloo.json
timeout -k 10 400 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -30 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
