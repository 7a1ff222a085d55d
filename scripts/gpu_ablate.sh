set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ablate
for K in 1 5; do
for F in 0 1 2 4 8 16 3 11 15; do
  HMC_FORCE_K=$K HMC_DEBUG_ABLATE=$F timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --steps 10 > gpurun_out/ablate/K${K}_F$F.log 2>&1 || exit $?
done
done
echo done
