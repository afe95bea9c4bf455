#!/bin/bash
# round 5 step 10: ping-pong pairs with the weight fragments read a step ahead; A/B of a build
# without SLP vectorisation of conv_pair (no packed-f32 VALU beside the other group's MFMAs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s10
mkdir -p $O
V=$PWD/bioengine_worker_amd/_native/variants/noslp/libbe_hip.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BE_HIP_LIB=$V timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/tests_noslp.log 2>&1 || { tail -30 $O/tests_noslp.log; exit 1; }
tail -1 $O/tests_noslp.log
timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases.jsonl 2> $O/pp_phases.err || { tail -20 $O/pp_phases.err; exit 1; }
BE_HIP_LIB=$V timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases_noslp.jsonl 2> $O/pp_phases_noslp.err || { tail -20 $O/pp_phases_noslp.err; exit 1; }
cut -c1-700 $O/pp_phases.jsonl $O/pp_phases_noslp.jsonl
timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs.jsonl 2> $O/pairs.err || { tail -20 $O/pairs.err; exit 1; }
BE_HIP_LIB=$V timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_noslp.jsonl 2> $O/pairs_noslp.err || { tail -20 $O/pairs_noslp.err; exit 1; }
grep '"pair"' $O/pairs.jsonl | sed "s/^/def /" | cut -c1-120
grep '"pair"' $O/pairs_noslp.jsonl | sed "s/^/noslp /" | cut -c1-120
for r in 1 2; do
  timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
  BE_HIP_LIB=$V timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
done
cut -c1-200 $O/head_ab.jsonl
