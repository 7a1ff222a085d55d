# Dev A/B (round 4), one box: NUTS c5 shape for HEAD (a), the U-turn check preload (b) and the
# release/acquire hand-off variant; then the c4 streaming bench at feeds of 6, 9, 10 launches.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_nuts.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pre_t.log 2>&1
HMC_LIB_PATH=understanding-hmc_amd/lib/libhmc_pre2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_nuts.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pre2_t.log 2>&1
for i in 1 2; do
  for L in libhmc_a libhmc_b libhmc_pre2 libhmc_relacq; do
    HMC_LIB_PATH=understanding-hmc_amd/lib/$L.so timeout -k 10 120 python scripts/dev/ab_nuts.py 65536 16 4 100 0.95 >> gpurun_out/nuts_ab.txt 2>&1
  done
done
for F in 6 9 10; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps $((F*2)) --warmup 2 --stream-feed $F > gpurun_out/c4_feed$F.json 2> gpurun_out/c4_feed$F.err
done
