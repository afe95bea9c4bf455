#!/bin/bash
# round 5 step 24: compact work-queue diffusion (diffuse_q_kernel) + the stem ping-pong with a
# 16-byte P region: tests, mask-stage A/B, per-call stem times, headline A/B, kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s24
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py tests/test_conv_pair.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 300 python3 -u tools/mask_bench.py --variants q1,q0 --reps 5 > $O/mask_ab.jsonl 2> $O/mask_ab.err || { tail -20 $O/mask_ab.err; exit 1; }
cat $O/mask_ab.jsonl
for st in 1 0; do
  BE_PAIR_PP_STEM=$st timeout -k 10 200 python3 tools/pair_bench.py --only-pairs --reps 5 > $O/pairs_stem$st.jsonl 2> $O/pairs_stem$st.err || { tail -20 $O/pairs_stem$st.err; exit 1; }
  python3 -c "
import json
for l in open('$O/pairs_stem$st.jsonl'):
    if '\"pair\"' in l:
        d=json.loads(l)
        if d['H']==224 and d['pair']=='down/0/0': print('stem_pp', $st, d['pair'], d['ms'], d['ms_min'])
"
done
for r in 1 2; do
  for cfg in "1 1" "1 0" "0 1" "0 0"; do
    set -- $cfg
    BE_DIFFUSE_QUEUE=$1 BE_PAIR_PP_STEM=$2 timeout -k 10 200 python -u tools/headline_ab.py > $O/head_q$1_s$2_$r.json 2>>$O/head_ab.err || exit 1
    echo "q$1 stem$2 $(cut -c1-100 $O/head_q$1_s$2_$r.json)"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
cd $R && python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "tiles_gather_kernel" --top 45 --width 120 > $O/kt_step_headline_b32.txt || exit 1
head -45 $O/kt_step_headline_b32.txt
