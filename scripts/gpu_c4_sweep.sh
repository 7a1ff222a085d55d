# c4 (D=1000, streaming diagnostics): iterations per launch x diagnostics feed cadence.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4s
for SF in "10 5" "20 2" "20 3" "40 1"; do
  set -- $SF
  timeout -k 10 300 python bench.py --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 --iters-per-step $1 --stream-feed $2 > gpurun_out/c4s/s$1_f$2.log 2>&1 || exit $?
done
for f in gpurun_out/c4s/*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"rhat_median": [0-9.e+]*' $f); done
echo done
