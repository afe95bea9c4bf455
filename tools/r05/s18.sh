#!/bin/bash
# round 5 step 18: Cellpose-SAM inference with the MFMA rel-pos kernel (default) vs fp32 einsums, and
# lin1 + GELU on the macro-tile GEMM (hyb) vs hipBLASLt + separate bias-GELU pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r05/s18
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for m in hip:lib torch:lib hip:hyb; do
    BE_CPSAM_RELPOS=${m%%:*} BE_CPSAM_INFER_GEMM=${m##*:} timeout -k 10 300 python3 tools/kt_driver.py cpsam_infer 4 2>/dev/null | grep cpsam | sed "s/^/$m /" | cut -c1-120 | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cpi -o t -- python3 $R/tools/kt_driver.py cpsam_infer 4 > $O/cpi.log 2>&1 || { tail $O/cpi.log; exit 1; }
cd $R
python3 - $O/cpi/t_kernel_stats.csv <<'PY' > $O/cpi_stats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"total kernel time {tot/1e6:.3f} ms over the whole run (warm-up included)")
for r in rows[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}% {int(r['Calls']):6d} calls  {r['Name'][:110]}")
PY
head -16 $O/cpi_stats.txt | cut -c1-150
rm -f $O/cpi/t_kernel_trace.csv
