# A/B timing of several builds of the same tree on one box (dev only, not a bench line):
#   bash scripts/dev/ab_libs.sh TAG "libA libB ..." [ab_nuts.py args]   (libX = understanding-hmc_amd/lib/libX.so)
set -e
TAG=$1; LIBS=$2; shift 2
mkdir -p gpurun_out
for L in $LIBS; do
  HMC_LIB_PATH=understanding-hmc_amd/lib/$L.so timeout -k 10 200 python scripts/dev/ab_nuts.py "$@" >> gpurun_out/ab_nuts_$TAG.txt 2>&1
done
