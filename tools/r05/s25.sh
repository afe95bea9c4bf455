#!/bin/bash
# round 5 step 25: mask stage: LDS-window flow following + one-wave hole filling (+ the diffusion
# queue of s24): tests, mask-stage A/B per component, headline A/B, kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s25
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 300 python3 -u tools/mask_bench.py --variants base,r04,fe:be_cp_follow_flows_xcd,fw0,q0 --reps 5 > $O/mask_ab.jsonl 2> $O/mask_ab.err || { tail -20 $O/mask_ab.err; exit 1; }
cut -c1-200 $O/mask_ab.jsonl
for r in 1 2; do
  for cfg in base follow_xcd fill_lds; do
    case $cfg in
      base) E="";;
      follow_xcd) E="BIOENGINE_FOLLOW_ENTRY=be_cp_follow_flows_xcd";;
      fill_lds) E="BE_FILL_WAVE=0";;
    esac
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
cd $R && python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "tiles_gather_kernel" --top 45 --width 120 > $O/kt_step_headline_b32.txt || exit 1
head -30 $O/kt_step_headline_b32.txt
