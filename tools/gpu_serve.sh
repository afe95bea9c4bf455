#!/bin/bash
# Serving-overhead session: traced c=1 run (per-stage spans from router and replica processes),
# then an untraced concurrency sweep.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/serve_trace
BE_REPLICA_PROFILE="$PWD/gpurun_out/serve_trace/replica_prof_{pid}.txt" BIOENGINE_TRACE=1 BIOENGINE_TRACE_FILE="$PWD/gpurun_out/serve_trace/trace_{pid}.json" \
  timeout -k 10 300 python -u tools/serve_bench.py --concurrency ${TRACE_CONC:-1} --seconds 4 > gpurun_out/serve_c1_traced.log 2>&1 || exit $?
python tools/trace_summary.py gpurun_out/serve_trace/*.json > gpurun_out/serve_trace_summary.jsonl
timeout -k 10 300 python -u tools/serve_bench.py --concurrency ${SERVE_CONC:-1,8,64} --seconds 5 > gpurun_out/serve_sweep.log 2>&1
