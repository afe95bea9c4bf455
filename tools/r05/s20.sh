#!/bin/bash
# round 5 step 20: served c=1 after the HWC staging + copy-back trims (s19 = before)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s20
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_app.py tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/latency_b1.py --host > $O/latency.log 2>&1 || { tail $O/latency.log; exit 1; }
tail -1 $O/latency.log | cut -c1-200
timeout -k 10 300 python -u tools/serve_bench.py --concurrency 1,64 --seconds 5 > $O/serve.log 2>&1 || { tail $O/serve.log; exit 1; }
grep '^{' $O/serve.log | cut -c1-220
BIOENGINE_TRACE=1 BIOENGINE_TRACE_FILE="$O/trace_{pid}.json" timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > $O/c1_trace.log 2>&1 || { tail $O/c1_trace.log; exit 1; }
python3 tools/trace_summary.py $O/trace_*.json > $O/trace_summary.jsonl
head -12 $O/trace_summary.jsonl
rm -f $O/trace_*.json
