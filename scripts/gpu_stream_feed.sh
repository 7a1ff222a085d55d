# Streaming diagnostics cadence: GPU stream tests, then c4 (D=1000, 131072 chains) with the
# diagnostics fed every step vs every 5 steps.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/feed
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/feed/pytest.log 2>&1 || exit $?
for F in ${FEEDS:-1 5}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 --stream-feed $F ${EXTRA:-} > gpurun_out/feed/c4_f$F${TAGX:-}.log 2>&1 || exit $?
done
for f in gpurun_out/feed/c4_*.log; do echo $f $(grep -o '"value": [0-9.e+]*\|"ess_per_s_median": [0-9.e+]*\|"rhat_median": [0-9.e+]*' $f); done
echo done
