#!/bin/bash
# round 4 step 2: igemm v2 (32-B swizzled halo, 4-wave 2-per-CU blocks) numerics + per-layer A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/s2_tests.log 2>&1 || { tail -40 gpurun_out/r04/s2_tests.log; exit 1; }
tail -2 gpurun_out/r04/s2_tests.log
timeout -k 10 300 python -u tools/igemm_bench.py > gpurun_out/r04/s2_bench.jsonl 2>&1; rc=$?
cat gpurun_out/r04/s2_bench.jsonl
exit $rc
