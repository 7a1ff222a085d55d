set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_stream.py -m gpu -q -rf -x > gpurun_out/pytest_stream.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_stream.log
exit $rc
