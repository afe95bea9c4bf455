#!/bin/bash
# round 5 step 34: served c=1 anatomy on the current tree: trace spans + cProfile of the replica child
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s34
mkdir -p $O
timeout -k 10 200 python tools/latency_b1.py --host > $O/latency_host.log 2>&1 || { tail $O/latency_host.log; exit 1; }
tail -1 $O/latency_host.log | cut -c1-200
BIOENGINE_TRACE=1 BIOENGINE_TRACE_FILE="$O/trace_{pid}.json" timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > $O/c1_trace.log 2>&1 || { tail $O/c1_trace.log; exit 1; }
grep '^{' $O/c1_trace.log | cut -c1-220
python3 tools/trace_summary.py $O/trace_*.json > $O/trace_summary.jsonl
head -16 $O/trace_summary.jsonl
rm -f $O/trace_*.json
BE_REPLICA_PROFILE="$O/replica_prof_{pid}.txt" timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > $O/serve_prof.log 2>&1 || { tail $O/serve_prof.log; exit 1; }
grep '^{' $O/serve_prof.log | cut -c1-200
ls $O
