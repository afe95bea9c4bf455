#!/bin/bash
# attention backward: dkv LDS-DMA (default now) + dq LDS-DMA variant; numerics, kernel A/B, train step
set -o pipefail
R=$PWD
O=$R/gpurun_out/s15
mkdir -p $O
V=$R/bioengine_worker_amd/_native/variants/dqdma/libbe_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py > $O/test_base.log 2>&1 || { tail -30 $O/test_base.log; exit 1; }
tail -1 $O/test_base.log
BE_HIP_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py > $O/test_dq.log 2>&1 || { tail -30 $O/test_dq.log; exit 1; }
tail -1 $O/test_dq.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py --iters 30 | sed 's/^/base /' >> $O/attn.jsonl || exit 1
  BE_HIP_LIB=$V timeout -k 10 120 python tools/attn_bench.py --iters 30 | sed 's/^/dqdma /' >> $O/attn.jsonl || exit 1
done
timeout -k 10 120 python tools/attn_bench.py --iters 30 --B 1 | sed 's/^/base /' >> $O/attn.jsonl || exit 1
BE_HIP_LIB=$V timeout -k 10 120 python tools/attn_bench.py --iters 30 --B 1 | sed 's/^/dqdma /' >> $O/attn.jsonl || exit 1
cat $O/attn.jsonl
for B in 8 1; do
  timeout -k 10 200 python tools/cpsam_train_bench.py --batch $B | sed 's/^/base /' >> $O/train.jsonl || exit 1
  BE_HIP_LIB=$V timeout -k 10 200 python tools/cpsam_train_bench.py --batch $B | sed 's/^/dqdma /' >> $O/train.jsonl || exit 1
done
cat $O/train.jsonl
cd /tmp && export TMPDIR=/tmp
BE_HIP_LIB=$V timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex "attn_bwd" --output-format csv -d $O/sq -o p -- python3 $R/tools/attn_bench.py --iters 2 > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/s15/sq/p_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: int(x) for c, x in v.items()})
PY
echo done
