#!/bin/bash
# the 8-rank cost model, shards timed forward and in reverse order
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sim}; mkdir -p $O
timeout -k 10 300 python -u tools/shard_sim.py --world 8 --reps 5 > $O/sim_fwd.json 2> $O/sim_fwd.err; rc=$?
echo "fwd rc=$rc"; cat $O/sim_fwd.json; [ $rc -eq 0 ] || { tail $O/sim_fwd.err; exit $rc; }
timeout -k 10 300 python -u tools/shard_sim.py --world 8 --reps 5 --rev --no-single > $O/sim_rev.json 2> $O/sim_rev.err; rc=$?
echo "rev rc=$rc"; cat $O/sim_rev.json; [ $rc -eq 0 ] || { tail $O/sim_rev.err; exit $rc; }
