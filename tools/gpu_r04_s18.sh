#!/bin/bash
# round 4 step 18: CPSAM batch-1 step kernel table with the per-shape auto GEMMs (s17 ran the
# library table; its summary used the old AdamW marker)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s18
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in auto; do
  BE_CPSAM_GEMM=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$g -o t -- python3 $R/tools/cpsam_train_bench.py --batch 1 --steps 8 > $O/kt_$g.log 2>&1 || { tail $O/kt_$g.log; exit 1; }
  python3 $R/tools/kt_steps.py $O/kt_$g/t_kernel_trace.csv --steps 4 --marker adamw2_kernel --top 40 --width 120 > $O/kt_table_$g.txt || exit 1
  echo "== $g"; head -3 $O/kt_table_$g.txt
done
