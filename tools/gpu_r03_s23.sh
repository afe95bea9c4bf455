#!/bin/bash
# fp8 GEMM: XS scales staged by LDS-DMA + hoisted epilogue operands; rowcol prefetch pipeline; relpos dq
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s23
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8.py tests/test_cpsam_train_gpu.py tests/test_cpsam_numerics_gpu.py -m gpu > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python tools/fp8_bench.py > $O/fp8_bench.jsonl 2>&1 || { tail $O/fp8_bench.jsonl; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/s23/fp8_bench.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(json.dumps(d))
PY
timeout -k 10 300 python tools/cpsam_train_bench.py --batch 1 8 --steps 20 > $O/train.jsonl 2>&1 || { tail $O/train.jsonl; exit 1; }
grep bench $O/train.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b8 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 3 > $O/b8.log 2>&1 || { tail $O/b8.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/b8/t_kernel_trace.csv --steps 4 --top 30 --width 100 > $O/b8_table.txt || exit 1
rm -f $O/b8/t_kernel_trace.csv
head -30 $O/b8_table.txt
echo done
