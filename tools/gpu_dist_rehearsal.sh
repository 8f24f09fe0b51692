# GPU box: the N > 1 code paths rehearsed on one GPU (2 ranks, gloo), their GPU tests, then (unless
# NO_N1=1) the N = 1 bench.  usage: bash tools/gpu_dist_rehearsal.sh <tag>
set -o pipefail
TAG=${1:-dist}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_dist_gpu.py tests/test_cli_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || { tail -40 $OUT/pytest_dist.log; exit 1; }
tail -3 $OUT/pytest_dist.log
# no launcher: bench.py --gpus 2 starts its own 2 ranks (torch.distributed.run as a child process)
MXMOE_DIST_BACKEND=gloo MXMOE_DIST_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --extras "" \
  > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail -30 $OUT/bench_n2_gloo.err; exit 1; }
cat $OUT/bench_n2_gloo.json
[ "${NO_N1:-0}" = 1 ] && exit 0
timeout -k 10 400 python bench.py > $OUT/bench_n1.json 2> $OUT/bench_n1.err || { tail -30 $OUT/bench_n1.err; exit 1; }
cat $OUT/bench_n1.json
