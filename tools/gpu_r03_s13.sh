#!/bin/bash
# attention backward counters (B=8 CPSAM shape): where the dq / dkv kernels' cycles go
set -o pipefail
R=$PWD
O=$R/gpurun_out/s13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex "attn_" --output-format csv -d $O/sq -o p -- python3 $R/tools/attn_bench.py --iters 2 > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES --kernel-trace --kernel-include-regex "attn_" --output-format csv -d $O/sq2 -o p -- python3 $R/tools/attn_bench.py --iters 2 > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, collections
for d in ("sq", "sq2"):
    rows = list(csv.DictReader(open(f"gpurun_out/s13/{d}/p_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(d, k, {c: round(x, 3) if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE") else int(x) for c, x in v.items()})
PY
echo done
