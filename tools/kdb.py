"""Per-kernel summary of rocprofv3 SQLite output (run_results.db, the default
output format): calls, average us, total ms, sorted by total.
  python tools/kdb.py gpurun_out/small6/b64/run_results.db [--top 25] [--csv out.csv]"""
import argparse
import csv
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=25)
ap.add_argument("--csv", default=None)
a = ap.parse_args()
con = sqlite3.connect(a.db)
rows = con.execute("select name, count(*), avg(end - start), sum(end - start) from kernels "
                   "group by name order by sum(end - start) desc").fetchall()
for name, n, avg, tot in rows[:a.top]:
    print(f"{n:6d}  avg {avg / 1e3:10.1f} us  tot {tot / 1e6:9.2f} ms  {name[:110]}")
if a.csv:
    with open(a.csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs", "TotalDurationNs"])
        for name, n, avg, tot in rows:
            w.writerow([name, n, avg, tot])
