#!/bin/bash
# round 4 step 28: after the native-pointer lifetime fix -- the IVF test alone, the full GPU suite,
# then the default 1-GPU bench on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s28
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_search_gpu.py > $O/search_test.log 2>&1 || { tail -30 $O/search_test.log; exit 1; }
tail -1 $O/search_test.log
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_full.log 2>&1 || { tail -30 $O/gpu_tests_full.log; exit 1; }
tail -1 $O/gpu_tests_full.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 1500 $O/bench_default.json
