"""Top kernels of a rocprofv3 --stats kernel_stats.csv (or every one under a
directory): total ms, calls, average us."""
import csv
import glob
import os
import sys

paths = []
for a in sys.argv[1:] or ["gpurun_out"]:
    paths += [a] if a.endswith(".csv") else glob.glob(os.path.join(a, "**", "*kernel_stats.csv"), recursive=True)
for p in paths:
    rows = sorted(csv.DictReader(open(p)), key=lambda r: -float(r["TotalDurationNs"]))
    print(p)
    for r in rows[:16]:
        print(f'  {float(r["TotalDurationNs"]) / 1e6:9.2f} ms  n={int(r["Calls"]):>5}  avg={float(r["AverageNs"]) / 1e3:9.1f} us'
              f'  {r["Name"][:100]}')
