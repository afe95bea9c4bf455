#!/bin/bash
# round 4 step 12: igemm on the deepest CPnet level by default (tests, engine A/B, headline), served
# search with cached-UTF-8 thumbnails and a replica-side profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm.py tests/test_conv_pair.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/cpnet_engine_ab.py --reps 10 --configs perlayer_deep,default,igemm_deep > $O/engine.jsonl 2>&1 || { tail -20 $O/engine.jsonl; exit 1; }
grep '^{' $O/engine.jsonl
timeout -k 10 300 python -u bench.py --no-extras --no-served --no-em --steps 20 --warmup 3 > $O/headline.log 2>&1 || { tail -20 $O/headline.log; exit 1; }
grep '^{' $O/headline.log | cut -c1-300
BE_REPLICA_PROFILE=$PWD/$O/replica_{pid}.prof.txt timeout -k 10 300 python -u tools/search_serve_bench.py --concurrency 1,64 --seconds 4 > $O/search_serve.log 2>&1 || { tail -20 $O/search_serve.log; exit 1; }
grep '^{' $O/search_serve.log | cut -c1-400
ls $O
