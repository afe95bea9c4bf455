#!/bin/bash
# round 4 step 32: cellpose GPU tests with the pooled follow_flows entry in the identity test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s32
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/test.log 2>&1; echo "rc=$?"; tail -2 $O/test.log
