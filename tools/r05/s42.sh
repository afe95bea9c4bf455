#!/bin/bash
# round 5 step 42: full GPU suite + the default bench on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s42
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -4 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log; tail -c 1500 $O/bench.log
exit $rc
