# Dev: one rocprofv3 --pmc pass over lag_bench (k_conv_series dispatches averaged), summarised in place:
#   bash scripts/dev/lagpmc.sh TAG LIB "COUNTERS" MODE N n D
set -e
TAG=$1; LIB=$2; P=$3; shift 3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/lagprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
HMC_LIB_PATH=$R/understanding-hmc_amd/lib/$LIB.so timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/$TAG -o run -- python3 $R/scripts/dev/lag_bench.py "$@" 2 > $O/$TAG.log 2>&1 || echo "pmc $TAG failed" >> $O/summary.txt
python3 - $O/$TAG $TAG >> $O/summary.txt <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])) if f else []:
    if "k_conv_series" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / len(v) for k, v in agg.items()})
PY
rm -rf $O/$TAG
