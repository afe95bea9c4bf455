#!/bin/bash
# round 5 step 45: the full GPU suite on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s45
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -4 $O/gpu_tests.log
exit $rc
