set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for K in 1 2 4 5 8; do
  HMC_FORCE_K=$K timeout -k 10 300 python bench.py --no-cpu-baseline --no-ess > gpurun_out/bench_K$K.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-ess --steps 10 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || exit $?
echo done
