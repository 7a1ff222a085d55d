# Dev A/B of lag-kernel builds (not a bench line): bash scripts/dev/lag_ab.sh "libA libB" "MODE N n D" ...
set -e
LIBS=$1; shift
for shape in "$@"; do
  for L in $LIBS; do
    HMC_LIB_PATH=understanding-hmc_amd/lib/$L.so timeout -k 10 200 python scripts/dev/lag_bench.py $shape 4 2>&1 | grep -v amdgpu.ids
  done
done
