#!/bin/bash
# round 5 step 22: the stem (8 -> 32 + projection) on the ping-pong kernel: conv_pair tests (incl.
# the forced ping-pong cases), phase stamps, per-call times and headline A/B vs BE_PAIR_PP_STEM=0
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s22
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases.jsonl 2> $O/pp_phases.err || { tail -20 $O/pp_phases.err; exit 1; }
for st in 1 0; do
  BE_PAIR_PP_STEM=$st timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_stem$st.jsonl 2> $O/pairs_stem$st.err || { tail -20 $O/pairs_stem$st.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/pp_phases.jsonl'):
    d=json.loads(l); print(d['call'], d['cin'], 'c2t', d['cycles_per_2tiles'], 'g0', d['work_g0'], 'g1', d['work_g1'])
for st in (1, 0):
  for l in open('$O/pairs_stem%d.jsonl' % st):
    if '\"pair\"' in l:
        d=json.loads(l)
        if d['H']==224: print('stem_pp', st, d['pair'], d['ms'], d['ms_min'])
" | cut -c1-330
for r in 1 2; do
  for st in 1 0; do
    BE_PAIR_PP_STEM=$st timeout -k 10 200 python -u tools/headline_ab.py > $O/head_stem${st}_$r.json 2>>$O/head_ab.err || exit 1
    echo "stem$st $(cut -c1-110 $O/head_stem${st}_$r.json)"
  done
done
