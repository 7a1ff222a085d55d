# Full round check on one MI355X: GPU parity tests, smoke(), the default bench line (with the
# CPU baseline), then the rocprofv3 evidence for the same workload.  Usage: bash scripts/gpu_round.sh TAG
set -u
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
bash scripts/profile.sh $TAG > gpurun_out/profile_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_traffic.log 2>&1 || exit $?
echo done
