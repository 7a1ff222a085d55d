# Dev A/B (round 4): NUTS c5 shape (65,536 chains, 32 iterations per launch) for builds
# libhmc_<name>.so through HMC_LIB_PATH (scripts/dev/ab_nuts.py), interleaved twice.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    HMC_LIB_PATH=understanding-hmc_amd/lib/libhmc_$v.so timeout -k 10 120 python scripts/dev/ab_nuts.py 65536 32 3 100 0.95 >> gpurun_out/nuts_lib_ab.txt 2>&1
  done
done
