# Dev A/B (round 4): one bench.py configuration with alternative builds swapped in place of
# libhmc.so on the box (bench.py refuses HMC_LIB_PATH), interleaved twice.
# usage: lib_ab.sh TAG "bench args" name1 name2 ...   (libhmc_<name>.so; "release" = libhmc.so)
set -e
TAG=$1; ARGS=$2; shift 2
L=understanding-hmc_amd/lib
mkdir -p gpurun_out
cp $L/libhmc.so $L/libhmc_release.so
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = release ]; then cp $L/libhmc_release.so $L/libhmc.so; else cp $L/libhmc_$v.so $L/libhmc.so; fi
    timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/ab_${TAG}_${v}_$i.json 2> gpurun_out/ab_${TAG}_${v}_$i.err
  done
done
cp $L/libhmc_release.so $L/libhmc.so
