set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for F in 0 32 64 128 256 480; do
  for L in 0 1; do
    HMC_DEBUG_ABLATE=$F HMC_DEBUG_L=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 --chains 32768 > gpurun_out/ab/F${F}_L$L.log 2>&1 || exit $?
  done
done
echo done
