# PMC passes over the one-pass lag kernel on the bench-shaped window (dev):
#   bash scripts/dev/prof_diag_pmc.sh TAG [tmax]
set -e
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/pmc_diag_$1"
TM="${2:-48}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export DIAG_KERNEL="$TM"
timeout -s KILL 200 rocprofv3 --kernel-include-regex k_conv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/p1" -o run -- \
  python3 "$R/scripts/dev/diag_time.py" 1048576 100 100 1 > "$OUT/p1.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-include-regex k_conv --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD \
  SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d "$OUT/p2" -o run -- \
  python3 "$R/scripts/dev/diag_time.py" 1048576 100 100 1 > "$OUT/p2.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-include-regex k_conv --pmc FETCH_SIZE --output-format csv -d "$OUT/p3" -o run -- \
  python3 "$R/scripts/dev/diag_time.py" 1048576 100 100 1 > "$OUT/p3.log" 2>&1
python3 "$R/scripts/pmc_summary.py" "$OUT" k_conv > "$OUT/summary.txt"
rm -rf "$OUT/p1" "$OUT/p2" "$OUT/p3"   # (the raw per-dispatch CSVs: summary only)
