#!/bin/bash
# round 5 step 1: sanity of the round-4 tree + advisor fixes on a fresh box: full GPU suite, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log; tail -c 3000 $O/bench.log | tail -2
exit $rc
