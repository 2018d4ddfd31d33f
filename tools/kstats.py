"""Summaries of bench runs: `kstats.py BENCH.json KERNEL_STATS.csv [label]` prints
the bench line's QPS / step / dominant kernel / roofline and the top kernels of
the rocprofv3 kernel_stats.csv; `kstats.py CSV...` prints each CSV."""
import csv
import json
import sys


def stats(path, top=14):
    for x in list(csv.DictReader(open(path)))[:top]:
        print(f"    {x['Name'][:66]:66s} {x['Calls']:>5s} avg_ms={float(x['AverageNs'])/1e6:9.4f} pct={float(x['Percentage']):6.2f}")


args = sys.argv[1:]
if args and args[0].endswith(".json"):
    r = json.load(open(args[0]))
    ro = r.get("roofline", {})
    print("variant", args[2] if len(args) > 2 else "-", "qps", round(r["value"]), "ms", round(r["ms_per_step"], 2),
          "key", ro.get("kernel"), round(ro.get("launch_ms", 0) or 0, 2), "frac", round(ro.get("frac", 0) or 0, 3),
          "verified", r.get("verified"), "replayed", r["config"].get("replayed_queries"))
    if len(args) > 1:
        stats(args[1])
else:
    for p in args:
        print("==", p)
        stats(p, 1000)
