#!/bin/bash
# round 4 step 10: headline kernel table (current default paths) and the compressed search tier at 58 M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s10
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/kt/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 40 --width 110 > $O/kt_table.txt || exit 1
rm -f $O/kt/t_kernel_trace.csv
head -30 $O/kt_table.txt
timeout -k 10 900 python -u tools/search_bench.py --n 58000000 --tiers compressed --refines 400,1000,2000 --reps 10 > $O/search58m.jsonl 2>&1 || { tail -20 $O/search58m.jsonl; exit 1; }
grep '^{' $O/search58m.jsonl | cut -c1-600
timeout -k 10 300 python -u tools/search_serve_bench.py --concurrency 64 --seconds 4 --profile gpurun_out/r04/s10/search_main_c64.prof.txt > $O/search_serve_prof.log 2>&1 || { tail -20 $O/search_serve_prof.log; exit 1; }
grep '^{' $O/search_serve_prof.log | cut -c1-300
