# Dev A/B (round 4): the c4 streaming bench with alternative builds swapped in place of libhmc.so
# on the box (bench.py refuses HMC_LIB_PATH), interleaved; usage: c4_lib_ab.sh name1 name2 ...
set -e
L=understanding-hmc_amd/lib
mkdir -p gpurun_out
cp $L/libhmc.so $L/libhmc_release.so
for i in 1 2; do
  for v in "$@"; do
    if [ "$v" = release ]; then cp $L/libhmc_release.so $L/libhmc.so; else cp $L/libhmc_$v.so $L/libhmc.so; fi
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 > gpurun_out/c4ab_${v}_$i.json 2> gpurun_out/c4ab_${v}_$i.err
  done
done
cp $L/libhmc_release.so $L/libhmc.so
