#!/bin/bash
# round 6, s1: gemm_8p correctness + perf vs gemm_mt / hipBLASLt on the CPSAM forward shapes
set -o pipefail
mkdir -p gpurun_out/r06/s1
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_8p.py > gpurun_out/r06/s1/test_gemm_8p.log 2>&1 || { tail -30 gpurun_out/r06/s1/test_gemm_8p.log; exit 1; }
tail -3 gpurun_out/r06/s1/test_gemm_8p.log
timeout -k 10 300 python -u tools/gemm_8p_bench.py > gpurun_out/r06/s1/bench.jsonl 2>&1
rc=$?
cat gpurun_out/r06/s1/bench.jsonl | grep -v amdgpu.ids
exit $rc
