# Round-6 A/B batch (dev, one box): lag pass r05 vs HEAD (c4 half, c3 window), NUTS hand-off
# relaxed vs release/acquire, bench lines (c4, D=300 NUTS diagonal and full cov_p), then the
# affected GPU tests.
set -e
L=understanding-hmc_amd/lib
O=gpurun_out/r06_ab1.txt
: > $O
for i in 1 2; do
  for lib in libhmc_r05.so libhmc.so; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/lag_bench.py half 131072 99 1000 5 >> $O 2>&1
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/lag_bench.py conv 262144 400 100 5 >> $O 2>&1
  done
done
for i in 1 2; do
  for lib in libhmc_relaxed.so libhmc.so; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 200 python scripts/dev/ab_nuts.py 65536 32 3 >> $O 2>&1
  done
done
B="timeout -k 10 400 python -u bench.py --no-cpu-baseline"
$B --config c4 --steps 10 --warmup 3 > gpurun_out/bench_r06d_c4_d1000.json 2> gpurun_out/bench_r06d_c4_d1000.err
$B --config c4 --steps 21 --warmup 1 > gpurun_out/bench_r06d_c4_d1000_s21.json 2> gpurun_out/bench_r06d_c4_d1000_s21.err
$B --sampler nuts --dim 300 --rho 0.5 --chains 16384 --iters-per-step 16 --steps 3 --warmup 1 > gpurun_out/bench_r06d_nuts_d300.json 2> gpurun_out/bench_r06d_nuts_d300.err
$B --sampler nuts --dim 300 --rho 0.5 --cov-p-rho 0.3 --chains 16384 --iters-per-step 16 --steps 3 --warmup 1 > gpurun_out/bench_r06d_nuts_d300_mass.json 2> gpurun_out/bench_r06d_nuts_d300_mass.err
timeout -k 10 1000 python -u -m pytest tests/test_gpu_convergence_sums.py tests/test_gpu_exact_ess.py tests/test_gpu_nuts.py tests/test_gpu_nuts_big.py tests/test_gpu_stream.py tests/test_integration_abi.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r06d.log 2>&1
