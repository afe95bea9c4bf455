#!/bin/bash
# round 5 step 19: served c=1 anatomy: direct batch-1 latency, then c=1 through the full stack with
# the trace spans on (router + replica processes write Chrome traces), summarised per span
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s19
mkdir -p $O
timeout -k 10 200 python tools/latency_b1.py --host > $O/latency.log 2>&1 || { tail $O/latency.log; exit 1; }
tail -3 $O/latency.log | cut -c1-200
timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > $O/c1_notrace.log 2>&1 || { tail $O/c1_notrace.log; exit 1; }
grep '^{' $O/c1_notrace.log | cut -c1-200
BIOENGINE_TRACE=1 BIOENGINE_TRACE_FILE="$O/trace_{pid}.json" timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > $O/c1_trace.log 2>&1 || { tail $O/c1_trace.log; exit 1; }
grep '^{' $O/c1_trace.log | cut -c1-200
python3 tools/trace_summary.py $O/trace_*.json > $O/trace_summary.jsonl
head -40 $O/trace_summary.jsonl
