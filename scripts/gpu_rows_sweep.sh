# Does the q_chain footprint (rows per chain) change the sampler's speed?  Same S, different K.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rows
for KS in "5 40" "20 40" "20 10" "80 10"; do
  set -- $KS
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps $1 --iters-per-step $2 --warmup 1 > gpurun_out/rows/k$1_s$2.log 2>&1 || exit $?
done
for f in gpurun_out/rows/*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"kernel_ms": [0-9.e+]*' $f | head -2); done
echo done
