#!/bin/bash
# round 5 step 17: ping-pong groups of 8 waves (two per SIMD per group, 128 VGPRs) vs 4 (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s17
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
for v in 4 8; do
  if [ $v = 4 ]; then L=$PWD/bioengine_worker_amd/_native/libbe_hip.so; else L=$VD/gw8/libbe_hip.so; fi
  BE_HIP_LIB=$L timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/tests_gw$v.log 2>&1 || { tail -30 $O/tests_gw$v.log; exit 1; }
  BE_HIP_LIB=$L timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases_gw$v.jsonl 2> $O/pp_phases_gw$v.err || { tail -20 $O/pp_phases_gw$v.err; exit 1; }
  BE_HIP_LIB=$L timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_gw$v.jsonl 2> $O/pairs_gw$v.err || { tail -20 $O/pairs_gw$v.err; exit 1; }
  echo "== gw$v $(tail -1 $O/tests_gw$v.log)"
  python3 -c "
import json,sys
for l in open('$O/pp_phases_gw$v.jsonl'):
    d=json.loads(l); print(d['call'], d['cin'], 'c2t', d['cycles_per_2tiles'], 'g0', d['work_g0'], 'g1', d['work_g1'])
for l in open('$O/pairs_gw$v.jsonl'):
    if '\"pair\"' in l:
        d=json.loads(l)
        if d['H']==224: print(d['pair'], d['ms'], d['ms_min'])
" | cut -c1-330
done
for r in 1 2; do
  for v in 4 8; do
    if [ $v = 4 ]; then L=$PWD/bioengine_worker_amd/_native/libbe_hip.so; else L=$VD/gw8/libbe_hip.so; fi
    BE_HIP_LIB=$L timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
  done
done
cut -c1-100 $O/head_ab.jsonl
