#!/bin/bash
# One GPU-box session: GPU tests, then the 1-GPU bench.  Stops at the first GPU fault / timeout.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
exit $rc
