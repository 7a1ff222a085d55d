set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dt
for DT in 0.1 0.0 1e-3 1e-6; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 --chains 32768 --dt $DT > gpurun_out/dt/dt$DT.log 2>&1 || exit $?
done
echo done
