"""Mean per-dispatch value of every PMC counter of one kernel across scripts/gpu_dense_pmc.sh passes.
Usage: python scripts/pmc_summary.py gpurun_out/<dir> <kernel-substring>"""
import collections
import csv
import glob
import sys

d, kern = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
