# Dense (c3) A/B: A = lib/ab/libhmc_A.so, B = the in-tree build (after the dense + NUTS GPU tests).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dab
timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_nuts.py -x -q --timeout 120 --timeout-method thread -k "dense or nuts" > gpurun_out/dab/pytest.log 2>&1 || exit $?
for r in 1 2; do
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --rho 0.95 --chains 262144 --steps 10 --warmup 2 "$@" > gpurun_out/dab/c3_${v}_$r.log 2>&1 || exit $?
done
done
for f in gpurun_out/dab/c3_*.log; do echo $f $(grep -o '"value": [0-9.e+]*' $f); done
echo done
