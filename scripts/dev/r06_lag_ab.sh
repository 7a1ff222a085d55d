# Round-6 dev A/B of the matrix-core lag pass (one box): libs given as arguments.
set -e
L=understanding-hmc_amd/lib
O=gpurun_out/r06_lag_ab.txt
: > $O
for i in 1 2; do
  for lib in "$@"; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/lag_bench.py half 131072 99 1000 5 >> $O 2>&1
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/lag_bench.py conv 262144 400 100 5 >> $O 2>&1
  done
done
