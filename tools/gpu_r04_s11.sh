#!/bin/bash
# round 4 step 11: compressed search tier at 58 M, served search with out-of-band strings (+ main-process
# profile), engine A/B with igemm on the deepest level only
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s11
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ivfpq.py tests/test_replica_wire.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/cpnet_engine_ab.py --reps 10 --configs perlayer_deep,igemm_L3,igemm_deep > $O/engine.jsonl 2>&1 || { tail -20 $O/engine.jsonl; exit 1; }
grep '^{' $O/engine.jsonl
timeout -k 10 300 python -u tools/search_serve_bench.py --concurrency 1,64 --seconds 4 --profile $O/search_main_c64.prof.txt > $O/search_serve.log 2>&1 || { tail -20 $O/search_serve.log; exit 1; }
grep '^{' $O/search_serve.log | cut -c1-400
timeout -k 10 900 python -u tools/search_bench.py --n 58000000 --tiers compressed --refines 400,1000,2000 --reps 10 > $O/search58m.jsonl 2>&1 || { tail -20 $O/search58m.jsonl; exit 1; }
grep '^{' $O/search58m.jsonl | cut -c1-600
