# SQ counters of the dense (c3) kernel (or PMC_BENCH_ARGS): MFMA busy vs VALU vs waits (separate --pmc passes).
set -u
R="$GRAFT_REPO_ROOT"
O=${PMC_OUT:-dpmc}
mkdir -p "$R/gpurun_out/$O"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/$O/counters.txt" 2>&1 || true
B="$R/bench.py --no-cpu-baseline --no-ess --steps 3 --warmup 1 ${PMC_BENCH_ARGS:---rho 0.95 --chains 262144}"
O=${PMC_OUT:-dpmc}
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/$O/p$i" -o run -- python3 $B > "$R/gpurun_out/$O/p$i.log" 2>&1 || exit $?
done
echo done
