#!/bin/bash
# s20 (batched colsums: numerics + CPSAM step) + fp8 GEMM bench kernel trace (hipBLASLt kernel names)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
bash tools/gpu_r03_s20.sh || exit 1
O=$R/gpurun_out/s21
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp8 -o t -- python3 $R/tools/fp8_bench.py > $O/fp8.log 2>&1 || { tail $O/fp8.log; exit 1; }
cd $R
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/s21/fp8/t_kernel_stats.csv")))
for r in rows[:40]:
    print(r["Name"][:150], r["Calls"], r["AverageNs"])
PY
rm -f $O/fp8/t_kernel_trace.csv
echo done
