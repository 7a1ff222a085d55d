# f64 MFMA issue-rate microbenchmark + kernel-trace profile of the dense (c3) bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dprof
timeout -k 10 120 ./scripts/ubench/mfma_f64 > gpurun_out/dprof/mfma_f64.txt 2>&1 || exit $?
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dprof/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-ess --rho 0.95 --chains 262144 --steps 10 --warmup 2 > "$R/gpurun_out/dprof/trace.log" 2>&1 || exit $?
echo done
