set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab2
for r in 1 2; do
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess > gpurun_out/ab2/fast_${v}_$r.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --fp-mode exact > gpurun_out/ab2/exact_${v}_$r.log 2>&1 || exit $?
done
done
echo done
