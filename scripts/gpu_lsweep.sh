set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lsweep
for L in 0 1 2 4 8 16; do
  HMC_DEBUG_ABLATE=$((1000+L)) timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 > gpurun_out/lsweep/L$L.log 2>&1 || exit $?
done
for N in 8192 32768; do
  HMC_DEBUG_ABLATE=1012 timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 --chains $N > gpurun_out/lsweep/N$N.log 2>&1 || exit $?
  HMC_DEBUG_ABLATE=1000 timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 --chains $N > gpurun_out/lsweep/N${N}_L0.log 2>&1 || exit $?
done
echo done
