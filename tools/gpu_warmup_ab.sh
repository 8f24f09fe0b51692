set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wu
timeout -k 10 300 python bench.py --no-scaling-sim --no-cpu-baseline > gpurun_out/wu/a.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-scaling-sim --no-cpu-baseline --warmup 300 --extras-warmup 300 > gpurun_out/wu/b.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --no-scaling-sim --no-cpu-baseline > gpurun_out/wu/c.json 2>/dev/null || exit 1
