# Dev A/B on one box: interleaved runs of several builds (HMC_LIB_PATH) of one kernel, each
# re-running its launches long enough for a stable clock.
# usage: ab_pair.sh wave|nuts|dense lib1 lib2 ...
set -e
L=understanding-hmc_amd/lib
K=$1; shift
case "$K" in
  wave)  ARGS="1048576 40 10 100 100 20" ;;
  nuts)  ARGS="" ;;
  dense) ARGS="" ;;
  *) echo "unknown kernel $K"; exit 2 ;;
esac
for i in 1 2; do
  for lib in "$@"; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python scripts/dev/ab_$K.py $ARGS
  done
done
