#!/bin/bash
# One GPU-box session: GPU tests, then the 1-GPU bench.  Stops at the first GPU fault / timeout.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) echo "pytest failed rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.log
tail -2 gpurun_out/bench.log
exit $rc
