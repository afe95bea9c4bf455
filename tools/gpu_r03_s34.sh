#!/bin/bash
# closing kernel tables on the final tree: headline step (32 images) and the CPSAM batch-8 step
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s34
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b8 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 3 > $O/b8.log 2>&1 || { tail $O/b8.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 40 --width 110 > $O/head_table.txt || exit 1
python3 tools/kt_steps.py $O/b8/t_kernel_trace.csv --steps 4 --top 40 --width 110 > $O/b8_table.txt || exit 1
rm -f $O/head/t_kernel_trace.csv $O/b8/t_kernel_trace.csv
head -3 $O/head_table.txt; head -3 $O/b8_table.txt
echo done
