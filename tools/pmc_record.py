"""write profiles/<name>.json PMC records from a pmc_summary run (stdin lines)"""
import json, sys, re
out, kernel, workload, rows, dims, batch, alg, note = sys.argv[1:9]
fetch = write = None
for line in open(sys.argv[9]):
    if kernel in line and "FETCH_SIZE" in line:
        fetch = float(re.search(r"'FETCH_SIZE': '([0-9.e+]+)'", line).group(1))
    if kernel in line and "WRITE_SIZE" in line:
        write = float(re.search(r"'WRITE_SIZE': '([0-9.e+]+)'", line).group(1))
rec = dict(workload=workload, corpus_rows=int(rows), dims=int(dims), query_batch=int(batch), kernel=kernel,
           FETCH_SIZE_KiB_per_launch=fetch, WRITE_SIZE_KiB_per_launch=write, gfx950_fetch_correction=2.0,
           hbm_bytes_per_launch=(2 * fetch + write) * 1024, algorithmic_bytes_per_launch=int(float(alg)), note=note,
           source="tools/pmc_traffic.sh (rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, separate runs); bytes = "
                  "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 per MI355X_MICROARCH.md HBM section")
json.dump(rec, open(out, "w"), indent=2)
print(json.dumps(rec))
