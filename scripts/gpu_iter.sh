set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --fp-mode exact > gpurun_out/bench_exact.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --dim 1000 --chains 16384 > gpurun_out/bench_d1000.log 2>&1 || exit $?
echo done
