# A/B on the default bench line (q_chain rows stored): A = lib/ab/libhmc_A.so, B = in-tree build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abs
for r in 1 2; do
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/abs/${v}_$r.log 2>&1 || exit $?
done
done
for f in gpurun_out/abs/*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $f | head -2); done
echo done
