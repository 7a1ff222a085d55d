set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/calib"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$R/scripts/calib_traffic.py" > "$OUT/f.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$R/scripts/calib_traffic.py" > "$OUT/w.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum --output-format csv -d "$OUT/ea" -o run -- python3 "$R/scripts/calib_traffic.py" > "$OUT/ea.log" 2>&1 || true
echo ok
