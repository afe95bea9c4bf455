#!/bin/bash
# round 5 step 13: kernel tables (rocprofv3 kernel trace) of the headline step, the CPSAM fine-tune
# step (batch 8), CPSAM inference and the ViT-B/14 fp8 embedder
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r05/s13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b8 -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 6 --warmup 3 > $O/b8.log 2>&1 || { tail $O/b8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vit -o t -- python3 $R/tools/kt_driver.py vit 10 > $O/vit.log 2>&1 || { tail $O/vit.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cpi -o t -- python3 $R/tools/kt_driver.py cpsam_infer 4 > $O/cpi.log 2>&1 || { tail $O/cpi.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 45 --width 120 > $O/head_table.txt || exit 1
python3 tools/kt_steps.py $O/b8/t_kernel_trace.csv --steps 4 --marker adamw2_kernel --top 40 --width 120 > $O/b8_table.txt || exit 1
head -30 $O/head_table.txt | cut -c1-140
head -12 $O/b8_table.txt | cut -c1-140
for d in vit cpi; do python3 - $O/$d/t_kernel_stats.csv <<'PY' > $O/${d}_stats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(f"total kernel time {tot/1e6:.3f} ms over the whole run (warm-up included)")
for r in rows[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {100*float(r['TotalDurationNs'])/tot:5.1f}% {int(r['Calls']):6d} calls  {r['Name'][:110]}")
PY
head -14 $O/${d}_stats.txt | cut -c1-140
done
rm -f $O/head/t_kernel_trace.csv $O/b8/t_kernel_trace.csv $O/vit/t_kernel_trace.csv $O/cpi/t_kernel_trace.csv
