#!/bin/bash
# round 5 step 8: ping-pong level-0 half-blocks (BE_PAIR_PP=1, default) vs the one-group kernel:
# numerics (pair tests, Cellpose / CPnet engine GPU tests), per-call pair timings, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s8
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py tests/test_cellpose_gpu.py tests/test_cpnet_engine_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for l in 0 1; do
  BE_PAIR_PP=$l timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_pp$l.jsonl 2> $O/pairs_pp$l.err || { tail -20 $O/pairs_pp$l.err; exit 1; }
  grep -v amdgpu.ids $O/pairs_pp$l.jsonl | sed "s/^/pp$l /" | cut -c1-160
done
for r in 1 2; do
  for l in 1 0; do
    BE_PAIR_PP=$l timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
  done
done
cut -c1-200 $O/head_ab.jsonl
