#!/bin/bash
# round 5 step 12: ping-pong pairs with bounds-free interior tiles (commit, halo issue, epilogue A)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s12
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py tests/test_cellpose_gpu.py tests/test_cpnet_engine_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases.jsonl 2> $O/pp_phases.err || { tail -20 $O/pp_phases.err; exit 1; }
cut -c1-700 $O/pp_phases.jsonl
timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs.jsonl 2> $O/pairs.err || { tail -20 $O/pairs.err; exit 1; }
grep '"pair"' $O/pairs.jsonl | cut -c1-120
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
done
cut -c1-150 $O/head_ab.jsonl
