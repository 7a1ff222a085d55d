# Dev: WRITE_SIZE per launch of the wave kernel for each build (one --pmc pass each).
set -e
L=understanding-hmc_amd/lib
R="${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for lib in "$@"; do
  OUT="$R/gpurun_out/abw_${lib%.so}"
  mkdir -p "$OUT"
  (cd /tmp && HMC_LIB_PATH=$R/$L/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o run -- \
     python3 "$R/scripts/dev/ab_wave.py" 1048576 40 3 100 100 1 > "$OUT/log" 2>&1)
  python3 scripts/pmc_summary.py "$OUT" "k_wave" > "$OUT/summary.txt"
done
