set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_drivers.py -m gpu -q -rf -x > gpurun_out/pytest_drv.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_drv.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python drivers/cases.py 1c 3c --seed 0 > gpurun_out/cases.log 2>&1 || exit $?
timeout -k 10 600 python drivers/cases.py 3c --seed 0 --chains 65536 --rng philox --fp-mode fast >> gpurun_out/cases.log 2>&1 || exit $?
echo done
