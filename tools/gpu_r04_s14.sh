#!/bin/bash
# round 4 step 14: ViT qkv GEMM A/B, fp8 GPU tests, then the full 1-GPU bench on the round-4 defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s14
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fp8.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/vit_qkv_ab.py > $O/vit_qkv_ab.jsonl 2>&1 || { tail -20 $O/vit_qkv_ab.jsonl; exit 1; }
grep '^{' $O/vit_qkv_ab.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-3000
