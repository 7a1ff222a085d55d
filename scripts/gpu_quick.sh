set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --fp-mode exact > gpurun_out/bench_exact.log 2>&1 || exit $?
echo done
