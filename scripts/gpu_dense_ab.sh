# Dense (c3) A/B on one build: A = chain-ordered tiles, B = L-ordered tiles (after the dense GPU tests).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dab
timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -k "dense" > gpurun_out/dab/pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --rho 0.95 --chains 262144 --steps 10 --warmup 2 --no-order-tiles > gpurun_out/dab/c3_A.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --rho 0.95 --chains 262144 --steps 10 --warmup 2 > gpurun_out/dab/c3_B.log 2>&1 || exit $?
grep -h -o '"value": [0-9.e+]*\|"frac": [0-9.e+]*' gpurun_out/dab/c3_*.log
echo done
