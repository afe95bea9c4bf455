#!/bin/bash
# round 5 step 36: follow-flows LDS window with an odd row stride (bank conflicts): tests, mask
# stage time, PMC pass on the mask kernels, headline + batch-1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/s36
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 200 python3 -u tools/mask_bench.py --variants base --reps 5 > $O/mask.jsonl 2> $O/mask.err || { tail $O/mask.err; exit 1; }
cut -c1-120 $O/mask.jsonl
for r in 1 2; do
  timeout -k 10 200 python -u tools/headline_ab.py > $O/head_$r.json 2>>$O/head_ab.err || exit 1
  echo "head $(cut -c1-100 $O/head_$r.json)"
done
timeout -k 10 200 python3 tools/latency_b1.py --iters 30 > $O/b1.json 2>/dev/null || exit 1
cat $O/b1.json
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/masks -o p -- python3 $R/tools/mask_bench.py --variants base --reps 2 > $O/masks_pmc.log 2>&1 || { tail $O/masks_pmc.log; exit 1; }
cd $R && python3 tools/pmc_summary.py $O/masks/p_counter_collection.csv --top 6 > $O/masks_summary.txt || exit 1
grep -A10 follow_flows $O/masks_summary.txt | head -12
python3 - <<'PY'
import csv, collections, os
O = os.environ.get("O") or "gpurun_out/r05/s36"
PY
rm -rf $O/masks
