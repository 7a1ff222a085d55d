# Samples board power and shader clock (rocm-smi, read-only) while the wave kernel runs for ~10 s.
set -e
OUT=gpurun_out/power_$1.log
: > $OUT
( for i in $(seq 1 24); do timeout 5 rocm-smi --showpower --showclocks >> $OUT 2>&1 || true; sleep 0.4; done ) &
SP=$!
timeout -k 10 120 python scripts/dev/ab_wave.py 1048576 40 10 100 ${2:-100} 50 >> $OUT 2>&1
wait $SP
