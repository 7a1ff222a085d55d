# Workgroup size of the K > 1 wave kernels: A = lib/ab/libhmc_A.so (256 threads), B = in-tree.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kb
timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > gpurun_out/kb/pytest.log 2>&1 || exit $?
for D in 200 400 1000; do
for v in A B; do
  if [ $v = A ]; then export HMC_LIB_PATH=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib/ab/libhmc_A.so; else unset HMC_LIB_PATH; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess --dim $D --chains 131072 --steps 5 --warmup 1 > gpurun_out/kb/d${D}_$v.log 2>&1 || exit $?
done
done
for f in gpurun_out/kb/d*.log; do echo $f $(grep -o '"value": [0-9.e+]*' $f); done
echo done
