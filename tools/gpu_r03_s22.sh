#!/bin/bash
# fp8 GEMM with hoisted epilogue operands: numerics + bench; then s20 (batched colsums) + hipBLASLt kernel names
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s22
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8.py -m gpu > $O/fp8_test.log 2>&1 || { tail -30 $O/fp8_test.log; exit 1; }
tail -1 $O/fp8_test.log
timeout -k 10 300 python tools/fp8_bench.py > $O/fp8_bench.jsonl 2>&1 || { tail $O/fp8_bench.jsonl; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/s22/fp8_bench.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print({k: v for k, v in d.items() if "by_tile" not in k})
PY
bash tools/gpu_r03_s20.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp8 -o t -- python3 $R/tools/fp8_bench.py > $O/fp8.log 2>&1 || { tail $O/fp8.log; exit 1; }
cd $R
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/s22/fp8/t_kernel_stats.csv")))
for r in rows[:40]:
    print(r["Name"][:150], r["Calls"], r["AverageNs"])
PY
rm -f $O/fp8/t_kernel_trace.csv
echo done
