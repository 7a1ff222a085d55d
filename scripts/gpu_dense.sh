set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_random.py -m gpu -q -rf -k "dense" > gpurun_out/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_dense.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --rho 0.95 --chains 262144 --steps 5 --warmup 1 > gpurun_out/bench_dense.log 2>&1 || exit $?
echo done
