# rocprofv3 kernel trace of convergence_stats on the bench-shaped window (dev): bash scripts/dev/prof_diag.sh TAG
set -e
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/prof_diag_$1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 "$R/scripts/dev/diag_time.py" 1048576 100 100 3 > "$OUT/run.log" 2>&1
