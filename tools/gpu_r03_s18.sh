#!/bin/bash
# attention backward with LDS-DMA dq + dkv: numerics, kernel times, train step, counters
set -o pipefail
R=$PWD
O=$R/gpurun_out/s18
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py tests/test_cpsam_numerics_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 120 python tools/attn_bench.py --iters 30 >> $O/attn.jsonl || exit 1
timeout -k 10 120 python tools/attn_bench.py --iters 30 --B 1 >> $O/attn.jsonl || exit 1
cat $O/attn.jsonl
timeout -k 10 300 python tools/cpsam_train_bench.py --batch 8 1 --steps 20 > $O/train.jsonl || exit 1
cat $O/train.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex "attn_" --output-format csv -d $O/sq -o p -- python3 $R/tools/attn_bench.py --iters 2 > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex "attn_" --output-format csv -d $O/sq1 -o p -- python3 $R/tools/attn_bench.py --iters 2 --B 1 > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, collections
for d in ("sq", "sq1"):
    rows = list(csv.DictReader(open(f"gpurun_out/s18/{d}/p_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(d, k, {c: int(x) for c, x in v.items()})
PY
echo done
