# Round-6 dev: c4 half-pass A/B plus one FETCH_SIZE/TA pass per library (libs as arguments).
set -e
L=$GRAFT_REPO_ROOT/understanding-hmc_amd/lib
O=$GRAFT_REPO_ROOT/gpurun_out/r06_lag_fetch.txt
: > $O
for i in 1 2; do
  for lib in "$@"; do
    HMC_LIB_PATH=$L/$lib timeout -k 10 120 python $GRAFT_REPO_ROOT/scripts/dev/lag_bench.py half 131072 99 1000 5 >> $O 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  rm -rf /tmp/lf
  HMC_LIB_PATH=$L/$lib timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TA_BUSY_avr --output-format csv -d /tmp/lf -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/lag_bench.py half 131072 99 1000 2 > /tmp/lf.log 2>&1
  python3 - /tmp/lf $lib >> $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "k_conv_mfma" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / len(v) for k, v in agg.items()})
PY
done
