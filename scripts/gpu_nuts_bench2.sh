set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for S in 2 8; do
timeout -k 10 300 python bench.py --sampler nuts --rho 0.95 --chains 65536 --iters-per-step $S --steps 3 --warmup 1 --no-cpu-baseline --no-ess > gpurun_out/bench_nuts_S$S.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --sampler nuts --rho 0.95 --chains 16384 --iters-per-step 2 --steps 3 --warmup 1 --no-cpu-baseline --no-ess > gpurun_out/bench_nuts_small.log 2>&1 || exit $?
echo done
