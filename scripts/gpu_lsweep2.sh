set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ls2
for L in 0 1 6 12 19; do
  HMC_DEBUG_L=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 > gpurun_out/ls2/L$L.log 2>&1 || exit $?
done
HMC_DEBUG_ABLATE=256 timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 > gpurun_out/ls2/nornd.log 2>&1 || exit $?
HMC_DEBUG_ABLATE=64 timeout -k 10 120 python bench.py --no-cpu-baseline --no-ess --steps 5 > gpurun_out/ls2/nostore.log 2>&1 || exit $?
cd /tmp; export TMPDIR=/tmp; R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$R/gpurun_out/ls2/pmc" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-ess --steps 3 --warmup 1 > "$R/gpurun_out/ls2/pmc.log" 2>&1 || exit $?
echo done
