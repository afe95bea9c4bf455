#!/bin/bash
# round 4 step 8: ping-pong GEMM / conv kernel: numerics, A/B bench, then the CPSAM GEMM-backend A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gemm_pp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/s8_tests.log 2>&1 || { tail -40 gpurun_out/r04/s8_tests.log; exit 1; }
tail -2 gpurun_out/r04/s8_tests.log
timeout -k 10 400 python -u tools/pp_bench.py --reps 10 > gpurun_out/r04/s8_pp.jsonl 2>&1 || { tail -20 gpurun_out/r04/s8_pp.jsonl; exit 1; }
grep '^{' gpurun_out/r04/s8_pp.jsonl
for g in lib auto; do
  BE_CPSAM_GEMM=$g timeout -k 10 300 python -u tools/cpsam_train_bench.py --batch 1 8 --steps 20 > gpurun_out/r04/s8_cpsam_$g.jsonl 2>&1 || { tail -20 gpurun_out/r04/s8_cpsam_$g.jsonl; exit 1; }
  grep '^{' gpurun_out/r04/s8_cpsam_$g.jsonl | cut -c1-400
done
