#!/bin/bash
# kernel stats of the C4 bench with the BQ fast path on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-bqprof}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --workload bq --option bq_fast=${2:-1} --no-cpu-baseline --steps 3 --warmup 1 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r["Calls"].rjust(6), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Name"][:90])
PY
