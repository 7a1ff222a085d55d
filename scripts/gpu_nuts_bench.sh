set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --sampler nuts --rho 0.95 --chains 65536 --iters-per-step 2 --steps 5 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_nuts.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --rho 0.95 --chains 262144 --iters-per-step 10 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dense.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nuts -o run -- python bench.py --sampler nuts --rho 0.95 --chains 65536 --iters-per-step 2 --steps 3 --warmup 1 --no-cpu-baseline --no-ess > gpurun_out/prof_nuts.log 2>&1 || exit $?
echo done
