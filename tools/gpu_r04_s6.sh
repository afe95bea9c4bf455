#!/bin/bash
# round 4 step 6: bf16 GEMM wave-tile configurations (8 waves of 64x64 vs 4 waves of 128x64 / 64x128)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gemm_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/s6_tests.log 2>&1 || { tail -40 gpurun_out/r04/s6_tests.log; exit 1; }
tail -2 gpurun_out/r04/s6_tests.log
timeout -k 10 400 python -u tools/gemm_bf16_bench.py --cfgs 0,1,2,3 --reps 10 > gpurun_out/r04/s6_gemm.jsonl 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r04/s6_gemm.jsonl
exit $rc
