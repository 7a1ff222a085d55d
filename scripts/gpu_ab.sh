# Same-box A/B of two libhmc.so builds on the bench workload: A = lib/ab/libhmc_A.so (baseline),
# B = the in-tree build.  Usage: bash scripts/gpu_ab.sh [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for r in 1 2; do
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess "$@" > gpurun_out/ab/fast_${v}_$r.log 2>&1 || exit $?
done
done
grep -h -o '"value": [0-9.e+]*' gpurun_out/ab/fast_*_*.log
echo done
