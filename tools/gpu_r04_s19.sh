#!/bin/bash
# round 4 step 19: CPSAM step with each parameter group's AdamW inside the graph on a side stream,
# against the flat update after the replay; the side-stream update's block cap swept
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s19
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
(cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py -k overlapped > $O/test.log 2>&1) || { tail $O/test.log; exit 1; }
timeout -k 10 200 python3 $R/tools/cpsam_train_bench.py --batch 1 8 --steps 20 --overlap-adamw 0 >> $O/ab.jsonl 2> $O/err0.log || exit 1
for cap in 256 64 32; do
  BE_ADAMW_BG_BLOCKS=$cap timeout -k 10 200 python3 $R/tools/cpsam_train_bench.py --batch 1 8 --steps 20 --overlap-adamw 1 >> $O/ab.jsonl 2> $O/err$cap.log || exit 1
done
timeout -k 10 200 python3 $R/tools/cpsam_train_bench.py --batch 1 8 --steps 20 --overlap-adamw 0 >> $O/ab.jsonl 2>> $O/err0.log || exit 1
cat $O/ab.jsonl
