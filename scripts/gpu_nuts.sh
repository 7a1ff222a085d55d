set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_nuts.py -m gpu -q -rf -x > gpurun_out/pytest_nuts.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_nuts.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --deselect tests/test_gpu_nuts.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
exit $rc
