#!/bin/bash
# round 4 step 1: implicit-GEMM conv numerics + per-layer A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm.py tests/test_conv_gpu.py tests/test_conv_pair.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/s1_tests.log 2>&1 || { tail -40 gpurun_out/r04/s1_tests.log; exit 1; }
tail -3 gpurun_out/r04/s1_tests.log
timeout -k 10 300 python -u tools/igemm_bench.py > gpurun_out/r04/s1_bench.jsonl 2>&1; rc=$?
cat gpurun_out/r04/s1_bench.jsonl
exit $rc
