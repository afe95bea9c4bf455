#!/bin/bash
# Batch-1 latency anatomy: wall p50, then rocprofv3 kernel stats of the same loop.
set -o pipefail
mkdir -p gpurun_out/prof_b1
timeout -k 10 300 python3 tools/latency_b1.py > gpurun_out/prof_b1/latency.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/latency_b1.py --host >> gpurun_out/prof_b1/latency.log 2>&1 || exit $?
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b1 -o b1 -- python3 $R/tools/latency_b1.py --iters 30 > $R/gpurun_out/prof_b1/prof_stdout.log 2>&1
