"""Condense a `scripts/gpu.sh prof` run into profiles/<tag>_*.{csv,json} (committed evidence).

HBM bytes per launch of the hot kernel = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B), the x2 being the
gfx950 correction for wide coalesced reads (MI355X_MICROARCH.md §HBM).  Only the timed launches
(the last `steps` dispatches of the hot kernel) are averaged.  The entry is keyed by the launch
shape the bench line reports (roofline.shape), and bench.py attaches it to a line only when that
line has the same shape."""
import csv
import glob
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
HOT = ("k_wave_iters", "k_random_iters", "k_dense_iters", "k_nuts_iters")


def one(pattern):
    f = sorted(glob.glob(os.path.join(out, pattern), recursive=True))
    return f[0] if f else None


def bench_line(logname):
    """The bench JSON line printed during a profiled run."""
    try:
        for line in open(os.path.join(out, logname)):
            if line.startswith("{") and '"metric"' in line:
                return json.loads(line)
    except OSError:
        pass
    return None


line = bench_line("trace.log") or bench_line("fetch.log")
steps = line["steps"] if line else 10
summary = {"tag": tag, "bench_line": line}
stats = one("trace/**/run_kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    hot = [r for r in rows if any(h in r["Name"] for h in HOT)]
    if hot:
        h = max(hot, key=lambda r: float(r["TotalDurationNs"]))
        summary["hot_kernel"] = h["Name"]
        summary["hot_avg_ns"] = float(h["AverageNs"])
        summary["hot_calls"] = int(h["Calls"])


def pmc(sub, name):
    f = one(f"{sub}/**/run_counter_collection.csv")
    if not f:
        return None
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == name and any(h in r["Kernel_Name"] for h in HOT)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    vals = [float(r["Counter_Value"]) for r in rows][-steps:]
    return sum(vals) / len(vals) if vals else None


fetch_kb, write_kb = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
if fetch_kb is not None and write_kb is not None:
    summary["fetch_size_kb"] = fetch_kb
    summary["write_size_kb"] = write_kb
    summary["bytes_per_launch"] = (2.0 * fetch_kb + write_kb) * 1024.0
sq = {}
f = one("sq/**/run_counter_collection.csv")
if f:
    agg = {}
    for r in csv.DictReader(open(f)):
        if any(h in r["Kernel_Name"] for h in HOT):
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    sq = {k: sum(v[-steps:]) / len(v[-steps:]) for k, v in agg.items()}
    summary["sq"] = sq
json.dump(summary, open(os.path.join(prof, f"{tag}_profile_summary.json"), "w"), indent=1)

shape = (line or {}).get("roofline", {}).get("shape") or (line or {}).get("memory", {}).get("shape")
if "bytes_per_launch" in summary and shape:
    path = os.path.join(prof, "pmc_traffic.json")
    try:
        entries = json.load(open(path))
        entries = entries if isinstance(entries, list) else []
    except (OSError, ValueError):
        entries = []
    entries = [e for e in entries if e.get("shape") != shape]
    entries.append({"shape": shape, "bytes_per_launch": summary["bytes_per_launch"],
                    "source": f"profiles/{tag}_profile_summary.json", "kernel": summary.get("hot_kernel")})
    json.dump(entries, open(path, "w"), indent=1)
print(json.dumps({k: v for k, v in summary.items() if k != "bench_line"}, indent=1))
