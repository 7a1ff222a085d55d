# Iterations fused per launch (bench --iters-per-step) on the default D=100 workload.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/isweep
for S in 10 20 40; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --iters-per-step $S --steps 10 > gpurun_out/isweep/noess_s$S.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline --iters-per-step $S --steps 10 > gpurun_out/isweep/store_s$S.log 2>&1 || exit $?
done
for f in gpurun_out/isweep/*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"ess_per_s_median": [0-9.e+]*' $f); done
echo done
