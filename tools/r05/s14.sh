#!/bin/bash
# round 5 step 14: ping-pong phase placement variants (PP_VAR: 1 = residual issued in P3, 2 = next
# halo issued after the P5 stores, 4 = no s_setprio on the MFMA phases): phases + per-call timings
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s14
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 1 2 4; do
  if [ $v = 0 ]; then L=$PWD/bioengine_worker_amd/_native/libbe_hip.so; else L=$VD/ppv$v/libbe_hip.so; fi
  BE_HIP_LIB=$L timeout -k 10 120 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py -k "kernel_matches or head" > $O/tests_v$v.log 2>&1 || { tail -30 $O/tests_v$v.log; exit 1; }
  BE_HIP_LIB=$L timeout -k 10 200 python3 tools/pp_phase_profile.py > $O/pp_phases_v$v.jsonl 2> $O/pp_phases_v$v.err || { tail -20 $O/pp_phases_v$v.err; exit 1; }
  BE_HIP_LIB=$L timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_v$v.jsonl 2> $O/pairs_v$v.err || { tail -20 $O/pairs_v$v.err; exit 1; }
  echo "== v$v $(tail -1 $O/tests_v$v.log)"
  python3 -c "
import json,sys
for l in open('$O/pp_phases_v$v.jsonl'):
    d=json.loads(l); print(d['call'], d['cin'], 'c2t', d['cycles_per_2tiles'], 'g0', d['work_g0'], 'g1', d['work_g1'])
for l in open('$O/pairs_v$v.jsonl'):
    if '\"pair\"' in l:
        d=json.loads(l)
        if d['H']==224: print(d['pair'], d['ms'], d['ms_min'])
" | cut -c1-330
done
