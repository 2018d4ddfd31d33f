"""Summarise rocprofv3 --pmc CSVs for the main kernels (per dispatch)."""
import collections, csv, glob, os, sys
root = sys.argv[1]
for path in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k, v in agg.items():
        if not any(s in k for s in ("mfma_select", "gemv_select", "exact_rows", "bq_", "pq_", "hamming_scan", "qs_", "q8_", "blk_", "rq")):
            continue
        n = len(disp[k])
        ms = sum(disp[k].values()) / n
        print(os.path.basename(os.path.dirname(path)), k, f"n={n} ms={ms:.2f}",
              {c: f"{x / n:.4g}" for c, x in sorted(v.items())})
