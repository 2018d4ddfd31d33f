#!/bin/bash
# round-6 closing benches: every workload through bench.py (C3 also under
# rocprofv3 kernel stats), one JSON line each under gpurun_out/<tag>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-final6}; mkdir -p $O
run() {  # name, bench args
    local n=$1; shift
    timeout -k 10 420 python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err; local rc=$?
    echo "$n rc=$rc"; tail -c 600 $O/bench_$n.json
    [ $rc -eq 0 ] || { tail -5 $O/bench_$n.err; exit $rc; }
}
run c3
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_c3_prof.json 2> $O/bench_c3_prof.err || { tail -5 $O/bench_c3_prof.err; exit 1; }
echo "c3 prof ok"
run c2 --workload c2
run c1 --workload c1
run bq --workload bq
run pq --workload pq
run rq8 --workload rq8
run rq1 --workload rq1
