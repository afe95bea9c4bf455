#!/bin/bash
# Serving tail-latency session: c=64 with the GC policy off / on (A/B), then a c=64 run with the
# replica's and the router process's cProfile.  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out/serve_tail
BIOENGINE_GC_TUNE=0 timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1,64 --seconds 6 > gpurun_out/serve_tail/gc_off.log 2>&1 || exit $?
BIOENGINE_GC_TUNE=1 timeout -k 10 240 python -u tools/serve_bench.py --concurrency 1,64 --seconds 6 > gpurun_out/serve_tail/gc_on.log 2>&1 || exit $?
BE_REPLICA_PROFILE="$PWD/gpurun_out/serve_tail/replica_prof_{pid}.txt" timeout -k 10 240 python -u tools/serve_bench.py --concurrency 64 --seconds 6 --profile gpurun_out/serve_tail/router_prof.txt > gpurun_out/serve_tail/prof.log 2>&1
