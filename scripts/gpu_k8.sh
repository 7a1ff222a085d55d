# K=8 wave kernel (D=1000): 2 waves/SIMD (HMC_K8_W2) vs 3 waves/SIMD, sampler only.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/k8
timeout -k 10 300 python -u -m pytest tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -k "wave" > gpurun_out/k8/pytest.log 2>&1 || exit $?
for r in 1 2; do
  HMC_K8_W2=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --dim 1000 --chains 131072 --steps 10 --warmup 2 > gpurun_out/k8/w2_$r.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ess --dim 1000 --chains 131072 --steps 10 --warmup 2 > gpurun_out/k8/w3_$r.log 2>&1 || exit $?
done
for f in gpurun_out/k8/w*.log; do echo $f $(grep -o '"value": [0-9.e+]*' $f); done
echo done
