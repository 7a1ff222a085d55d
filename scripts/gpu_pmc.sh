set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
BENCH="$R/bench.py --no-cpu-baseline --no-ess --steps 3 --warmup 1"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python3 $BENCH > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc" >> "$R/gpurun_out/pmc/status.txt"
  if [ $rc -ne 0 ] && [ $i -le 4 ]; then exit $rc; fi
done
echo done
