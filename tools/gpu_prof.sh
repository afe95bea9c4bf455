#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (no extras).  Output under gpurun_out/prof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 --no-extras ${PROF_ARGS:-} > gpurun_out/prof/bench_stdout.log 2>&1
rc=$?
echo "prof rc=$rc" >> gpurun_out/prof/bench_stdout.log
find gpurun_out/prof -name "*stats*" | head >> gpurun_out/prof/bench_stdout.log
exit $rc
