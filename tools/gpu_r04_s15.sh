#!/bin/bash
# round 4 step 15: the whole GPU test suite on the round-4 tree (what the driver runs at round end)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s15
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; rc=$?
tail -15 $O/gpu_tests.log
exit $rc
