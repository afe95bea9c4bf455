#!/bin/bash
# round 5 step 2: gemm_mt numerics (GPU tests) then the per-shape sweep against the library GEMM;
# the MX LayerNorm / fp8 tests, the ViT-L CPSAM inference engine test, the ViT qkv A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_mt.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u tools/gemm_mt_bench.py --table --rounds 5 > $O/sweep.jsonl 2>&1
rc=$?; echo "sweep rc=$rc" >> $O/sweep.jsonl; grep -v '"mt"' $O/sweep.jsonl | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_fp8.py tests/test_transformer_gpu.py tests/test_conv3d.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests2.log; tail -5 $O/tests2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/vit_qkv_ab.py > $O/vit_qkv_ab.jsonl 2>&1
rc=$?; cat $O/vit_qkv_ab.jsonl | tail -3
exit $rc
