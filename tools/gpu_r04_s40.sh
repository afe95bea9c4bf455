#!/bin/bash
# round 4 step 40: kernel tables of the final tree -- headline step (batch 32) and the CPSAM batch-8
# and batch-1 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s40
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b8 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 6 --warmup 3 > $O/b8.log 2>&1 || { tail $O/b8.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 45 --width 120 > $O/head_table.txt || exit 1
python3 tools/kt_steps.py $O/b8/t_kernel_trace.csv --steps 4 --marker adamw2_kernel --top 40 --width 120 > $O/b8_table.txt || exit 1
rm -f $O/head/t_kernel_trace.csv $O/b8/t_kernel_trace.csv
head -3 $O/head_table.txt; head -3 $O/b8_table.txt
