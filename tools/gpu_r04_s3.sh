#!/bin/bash
# round 4 step 3: igemm v2 conv + bf16 GEMM numerics and A/B benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py tests/test_gemm_bf16.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/s3_tests.log 2>&1 || { tail -40 gpurun_out/r04/s3_tests.log; exit 1; }
tail -2 gpurun_out/r04/s3_tests.log
timeout -k 10 240 python -u tools/igemm_bench.py > gpurun_out/r04/s3_conv.jsonl 2>&1 || { tail -20 gpurun_out/r04/s3_conv.jsonl; exit 1; }
cat gpurun_out/r04/s3_conv.jsonl
timeout -k 10 200 python -u tools/cpnet_engine_ab.py > gpurun_out/r04/s3_engine.jsonl 2>&1 || { tail -20 gpurun_out/r04/s3_engine.jsonl; exit 1; }
cat gpurun_out/r04/s3_engine.jsonl
timeout -k 10 240 python -u tools/gemm_bf16_bench.py > gpurun_out/r04/s3_gemm.jsonl 2>&1; rc=$?
cat gpurun_out/r04/s3_gemm.jsonl
exit $rc
