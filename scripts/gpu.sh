# One parameterised runner for every GPU-box job (replaces the round-1 one-off scripts).
#
#   bash scripts/gpu.sh test    TAG                 pytest -m gpu + smoke()
#   bash scripts/gpu.sh bench   TAG [bench args]    one bench.py line -> gpurun_out/bench_TAG.json
#   bash scripts/gpu.sh prof    TAG [bench args]    rocprofv3 kernel trace + stats, FETCH_SIZE and WRITE_SIZE
#                                                   (separate --pmc passes), SQ counters; summarise them
#                                                   into profiles/TAG_* afterwards, in the build container:
#                                                   python scripts/summarize_profile.py gpurun_out/prof_TAG TAG
#   bash scripts/gpu.sh pmc     TAG "CNT CNT ..." [bench args]   one extra --pmc pass (<= hardware limits)
#   bash scripts/gpu.sh configs TAG                 bench lines + kernel stats of BASELINE configs 3, 4, 5
#   bash scripts/gpu.sh round   TAG                 test, default bench, prof of the default bench
#   bash scripts/gpu.sh ubench                      build + run the micro-benchmarks in scripts/ubench
#
# Every GPU step runs under its own time limit and the steps are chained with && / exit on failure:
# after a fault, abort, timeout or hang nothing more runs on the GPU in this call.
set -u
CMD=${1:?usage: gpu.sh test|bench|prof|pmc|configs|round|ubench TAG [args]}
TAG=${2:-run}
shift 2 2>/dev/null || shift $#
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp

do_test() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || return $?
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
}

do_bench() {   # bench args...
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
}

do_prof() {    # bench args...
  local OUT="$R/gpurun_out/prof_$TAG"
  local ARGS="--no-cpu-baseline --steps 10 --warmup 2 $*"
  mkdir -p "$OUT"
  (cd /tmp &&
   timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
     python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
     python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
     python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 &&
   timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES \
     SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/sq" -o run -- \
     python3 "$R/bench.py" $ARGS > "$OUT/sq.log" 2>&1) || return $?
}

do_pmc() {     # "counters" bench args...
  local P=$1; shift
  local OUT="$R/gpurun_out/pmc_$TAG"
  mkdir -p "$OUT"
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT" -o run -- \
     python3 "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 2 "$@" > "$OUT/pmc.log" 2>&1) || return $?
  python3 scripts/pmc_summary.py "$OUT" "k_" > "$OUT/summary.txt"
}

do_configs() {
  local T=$TAG
  TAG=${T}_c3_dense;  do_bench --no-cpu-baseline --rho 0.95 --chains 262144 --steps 10 --warmup 2 || return $?
  TAG=${T}_c5_nuts;   do_bench --no-cpu-baseline --sampler nuts --rho 0.95 --chains 65536 --steps 5 --warmup 1 || return $?
  TAG=${T}_c4_d1000;  do_bench --no-cpu-baseline --dim 1000 --chains 131072 --stream-diag --steps 10 --warmup 2 || return $?
  TAG=${T}_c3_dense;  do_prof --rho 0.95 --chains 262144 || return $?
  TAG=${T}_c5_nuts;   do_prof --sampler nuts --rho 0.95 --chains 65536 --steps 5 --warmup 1 || return $?
  TAG=$T
}

do_ubench() {
  mkdir -p gpurun_out/ubench
  for f in scripts/ubench/*.hip; do
    b=gpurun_out/ubench/$(basename "$f" .hip)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o "$b" "$f" || return $?
    timeout -k 10 120 "$b" > "$b.txt" 2>&1 || return $?
  done
}

case "$CMD" in
  test) do_test ;;
  bench) do_bench "$@" ;;
  prof) do_prof "$@" ;;
  pmc) do_pmc "$@" ;;
  configs) do_configs ;;
  round) do_test && do_bench && do_prof ;;
  ubench) do_ubench ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
rc=$?
echo "gpu.sh $CMD $TAG rc=$rc"
exit $rc
