# NUTS (c5) A/B: A = lib/ab/libhmc_A.so, B = in-tree build, at 2 iterations per launch; then B at
# longer launches (lane utilisation vs iterations per launch).  NUTS GPU tests first.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/nab
timeout -k 10 300 python -u -m pytest tests/test_gpu_nuts.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nab/pytest.log 2>&1 || exit $?
C="--no-cpu-baseline --no-ess --sampler nuts --rho 0.95 --chains 65536"
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 200 python bench.py $C --iters-per-step 2 --steps 5 --warmup 1 > gpurun_out/nab/c5_${v}_s2.log 2>&1 || exit $?
done
unset HMC_LIB_PATH
for S in ${NUTS_S:-}; do
  timeout -k 10 300 python bench.py $C --iters-per-step $S --steps 3 --warmup 1 > gpurun_out/nab/c5_B_s$S.log 2>&1 || exit $?
done
for f in gpurun_out/nab/c5_*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"lane_utilisation": [0-9.e+]*\|"ms_per_step": [0-9.e+]*' $f); done
echo done
