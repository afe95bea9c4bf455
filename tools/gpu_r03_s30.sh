#!/bin/bash
# flat GELU forward pass vs the row-blocked one: numerics + CPSAM batch-8 A/B
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s30
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in 0 1 0 1; do
  BE_GELU_FWD_FLAT=$v timeout -k 10 200 python tools/cpsam_train_bench.py --batch 8 --steps 20 > $O/train_$v.jsonl 2>&1 || { tail $O/train_$v.jsonl; exit 1; }
  echo flat=$v $(grep bench $O/train_$v.jsonl | cut -c1-140)
done
echo done
