# Dev A/B on one box: interleaved runs of several builds of the wave kernel (HMC_LIB_PATH),
# each re-running its launches long enough for a stable clock.  usage: ab_pair.sh lib1 lib2 ...
set -e
L=understanding-hmc_amd/lib
for i in 1 2; do
  for lib in "$@"; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/ab_wave.py 1048576 40 10 100 100 20
  done
done
