set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --stream-diag > gpurun_out/bench_stream.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --stream-diag --dim 1000 --chains 131072 > gpurun_out/bench_c4.log 2>&1 || exit $?
echo done
