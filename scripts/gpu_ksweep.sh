set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ks
for K in 1 2 4 5 8 16; do
HMC_FORCE_K=$K timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 10 > gpurun_out/ks/K$K.log 2>&1 || exit $?
done
for K in 4 8 16; do
HMC_FORCE_K=$K timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 10 --chains 524288 > gpurun_out/ks/K${K}_big.log 2>&1 || exit $?
done
echo done
