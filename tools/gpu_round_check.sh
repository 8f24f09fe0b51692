set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1 || { tail -30 gpurun_out/pytest_r02a.log; exit 1; }
tail -3 gpurun_out/pytest_r02a.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02a.log 2>&1 || exit 1
bash tools/gpu_bench_profile.sh r02a --extras w8a8,w4a4,mixed,ds2_mixed
