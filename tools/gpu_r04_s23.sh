#!/bin/bash
# round 4 step 23: phase profile of the fused CPnet half-blocks (s_memtime-stamped diagnostic build),
# after the conv_pair numerics tests on the production build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s23
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 python3 tools/pair_phase_profile.py > $O/phases.jsonl 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
cat $O/phases.jsonl
# the final tree: full GPU suite, then the default 1-GPU bench
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_full.log 2>&1 || { tail -30 $O/gpu_tests_full.log; exit 1; }
tail -1 $O/gpu_tests_full.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 3000 $O/bench_default.json
