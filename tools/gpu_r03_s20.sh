#!/bin/bash
# batched colsums / bf16 column partials / slab sums: numerics, then the CPSAM step at batch 1 and 8
set -o pipefail
R=$PWD
O=$R/gpurun_out/s20
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py tests/test_cpsam_numerics_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python tools/cpsam_train_bench.py --batch 1 8 --steps 20 > $O/train.jsonl 2>&1 || { tail $O/train.jsonl; exit 1; }
grep bench $O/train.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 1 --steps 5 --warmup 3 > $O/b1.log 2>&1 || { tail $O/b1.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/b1/t_kernel_trace.csv --steps 4 --top 30 --width 100 > $O/b1_table.txt || exit 1
rm -f $O/b1/t_kernel_trace.csv
head -30 $O/b1_table.txt
echo done
