#!/bin/bash
# kernel trace of the simulated 8-rank step (tools/shard_sim.py), per-kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-simprof}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u tools/shard_sim.py --world 8 --reps 5 --no-single > $O/sim.json 2> $O/sim.err || { tail $O/sim.err; exit 1; }
cat $O/sim.json | tail -c 1500
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:30]:
    print(r["Calls"].rjust(6), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", ("%.1f" % (float(r["TotalDurationNs"]) / 1e6)).rjust(8), "ms", r["Name"][:90])
PY
