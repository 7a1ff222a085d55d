set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_nuts.py -m gpu -q -rf -x > gpurun_out/pytest_nuts.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_nuts.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for S in 2 8; do
timeout -k 10 300 python bench.py --sampler nuts --rho 0.95 --chains 65536 --iters-per-step $S --steps 3 --warmup 1 --no-cpu-baseline --no-ess > gpurun_out/bench_nuts_S$S.log 2>&1 || exit $?
done
echo done
