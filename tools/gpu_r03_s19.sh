#!/bin/bash
# kernel traces: CPSAM step at batch 8 and 1 (current tree), fp8 GEMM bench (our kernel vs hipBLASLt kernel names)
set -o pipefail
R=$PWD
O=$R/gpurun_out/s19
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b8 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 3 > $O/b8.log 2>&1 || { tail $O/b8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 1 --steps 5 --warmup 3 > $O/b1.log 2>&1 || { tail $O/b1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp8 -o t -- python3 $R/tools/fp8_bench.py > $O/fp8.log 2>&1 || { tail $O/fp8.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/b8/t_kernel_trace.csv --steps 4 --top 45 --width 110 > $O/b8_table.txt || exit 1
python3 tools/kt_steps.py $O/b1/t_kernel_trace.csv --steps 4 --top 45 --width 110 > $O/b1_table.txt || exit 1
head -30 $O/b8_table.txt; head -30 $O/b1_table.txt
rm -f $O/b8/t_kernel_trace.csv $O/b1/t_kernel_trace.csv
echo done
