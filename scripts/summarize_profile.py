"""Condense a scripts/profile.sh run into profiles/<tag>_*.{csv,json} (committed evidence).

HBM bytes per launch of the hot kernel = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B), the x2 being
the gfx950 correction for wide coalesced reads (MI355X_MICROARCH.md §HBM).  The hot kernel
reads only its state (q, E_prev) once per launch; its traffic is dominated by stores."""
import csv
import glob
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]
write_traffic_file = "--no-traffic-file" not in sys.argv[3:]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
HOT = ("k_wave_iters", "k_random_iters", "k_dense_iters", "k_nuts_iters")


def one(pattern):
    f = glob.glob(os.path.join(out, pattern), recursive=True)
    return f[0] if f else None


stats = one("trace/**/run_kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
summary = {"tag": tag}
if stats:
    rows = list(csv.DictReader(open(stats)))
    hot = [r for r in rows if any(h in r["Name"] for h in HOT)]
    if hot:
        h = max(hot, key=lambda r: float(r["TotalDurationNs"]))
        summary["hot_kernel"] = h["Name"]
        summary["hot_avg_ns"] = float(h["AverageNs"])
        summary["hot_calls"] = int(h["Calls"])


def pmc(sub, name, timed_only=True):
    """Mean of a PMC counter over the hot kernel's dispatches; the bench's warm-up launches
    (which store no q_chain rows) are dropped by keeping the last 10 dispatches (= --steps 10)."""
    f = one(f"{sub}/**/run_counter_collection.csv")
    if not f:
        return None
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == name and any(h in r["Kernel_Name"] for h in HOT)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    vals = [float(r["Counter_Value"]) for r in rows]
    if timed_only and len(vals) > 10:
        vals = vals[-10:]
    return sum(vals) / len(vals) if vals else None


fetch_kb, write_kb = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
if fetch_kb is not None and write_kb is not None:
    summary["fetch_size_kb"] = fetch_kb
    summary["write_size_kb"] = write_kb
    summary["bytes_per_launch"] = (2.0 * fetch_kb + write_kb) * 1024.0
sq = {}
for sub in ("sq", "sq2"):
    f = one(f"{sub}/**/run_counter_collection.csv")
    if f:
        agg = {}
        for r in csv.DictReader(open(f)):
            if any(h in r["Kernel_Name"] for h in HOT):
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        sq.update({k: sum(v) / len(v) for k, v in agg.items()})
if sq:
    summary["sq"] = sq
json.dump(summary, open(os.path.join(prof, f"{tag}_profile_summary.json"), "w"), indent=1)
if "bytes_per_launch" in summary and write_traffic_file:
    json.dump({"bytes_per_launch": summary["bytes_per_launch"], "source": f"profiles/{tag}_profile_summary.json",
               "kernel": summary.get("hot_kernel")},
              open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
