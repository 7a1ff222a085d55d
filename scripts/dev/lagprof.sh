# Dev: SQ counters of the lag kernel (one pass per counter set), summarised in place (the raw CSVs
# of the randn/AR set-up kernels are large): bash scripts/dev/lagprof.sh MODE N n D
# (KNAME selects the kernel: k_conv_series by default, k_conv_mfma for the matrix-core pass)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lagprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
export KNAME=${KNAME:-k_conv_series}
if [ "$KNAME" = "k_conv_mfma" ]; then
  SETS=("SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES"
        "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES"
        "FETCH_SIZE TA_BUSY_avr TA_BUSY_max")
else
  SETS=("SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU"
        "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_FLAT"
        "FETCH_SIZE TA_BUSY_avr TA_BUSY_max")
fi
for P in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 $R/scripts/dev/lag_bench.py "$@" 2 > $O/p$i.log 2>&1 || echo "pass $i failed" >> $O/summary.txt
  python3 - $O/p$i >> $O/summary.txt <<'PY'
import csv, glob, os, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])) if f else []:
    if os.environ["KNAME"] in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: sum(v) / len(v) for k, v in agg.items()})
PY
  rm -rf $O/p$i
done
