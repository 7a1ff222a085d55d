# rocprofv3 evidence for the bench workload: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE
# in separate PMC passes (MI355X_MICROARCH.md §HBM / rocprofv3 PMC slots).  Usage: bash scripts/profile.sh TAG
set -u
TAG=${1:-r01}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 10 --warmup 2"}   # default: the bench line's workload (q_chain rows stored)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/sq.log" 2>&1 || exit $?
if [ -n "${EXTRA_PMC:-}" ]; then
  timeout -k 10 600 rocprofv3 --pmc $EXTRA_PMC --output-format csv -d "$OUT/sq2" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/sq2.log" 2>&1 || exit $?
fi
cd "$R" && python3 scripts/summarize_profile.py "$OUT" "$TAG" ${NO_TRAFFIC_FILE:+--no-traffic-file}
