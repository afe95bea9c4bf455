#!/bin/bash
# round 4 step 21: per-shape GEMM choice timed on graph replays (kernel time, not launch overhead):
# test, then the CPSAM step with it against the library at batch 1 / 8, and the batch-1 kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s21
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_auto_gpu.py tests/test_transformer_gpu.py tests/test_cpsam_train_gpu.py tests/test_cpsam_numerics_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
cd /tmp && export TMPDIR=/tmp
for g in lib auto lib auto; do
  BE_CPSAM_GEMM=$g timeout -k 10 200 python3 $R/tools/cpsam_train_bench.py --batch 1 8 --steps 20 >> $O/ab.jsonl 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
done
# attention forward: 4-wave blocks (128 at batch 1) vs the new small-grid pick (2-wave, 256 blocks)
for nw in 4 0 4 0; do
  BE_ATTN_NW=$nw timeout -k 10 200 python3 $R/tools/cpsam_train_bench.py --batch 1 --steps 30 > $O/attn_nw$nw.json 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
  echo "attn nw=$nw $(grep -o '"ms_per_step": [0-9.]*' $O/attn_nw$nw.json)" | tee -a $O/attn_ab.txt
done
BE_CPSAM_GEMM=auto timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_auto -o t -- python3 $R/tools/cpsam_train_bench.py --batch 1 --steps 8 > $O/kt_auto.log 2>&1 || { tail $O/kt_auto.log; exit 1; }
python3 $R/tools/kt_steps.py $O/kt_auto/t_kernel_trace.csv --steps 4 --marker adamw2_kernel --top 40 --width 120 > $O/kt_table_auto.txt || exit 1
rm -f $O/kt_auto/t_kernel_trace.csv
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d = json.loads(l); print(d['gemm'], d['batch'], d['ms_per_step'], d.get('gemm_choices', {}).get('hip'), d.get('gemm_choices', {}).get('lib'))
"
