# Dev: one PMC pass over scripts/dev/ab_wave.py for the default and an alternative build.
# usage: bash scripts/dev/pmc_ab.sh TAG ALT_LIB "COUNTERS" [ab args]
set -u
TAG=$1; ALT=$2; P=$3; shift 3
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/pmcab_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$OUT/main" -o run -- python3 "$R/scripts/dev/ab_wave.py" "$@" > "$OUT/main.log" 2>&1 || exit $?
HMC_LIB_PATH="$R/$ALT" timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$OUT/alt" -o run -- python3 "$R/scripts/dev/ab_wave.py" "$@" > "$OUT/alt.log" 2>&1 || exit $?
cd "$R" && for v in main alt; do echo "== $v"; python3 scripts/pmc_summary.py "$OUT/$v" k_wave; grep "lf/s" "$OUT/$v.log"; done
