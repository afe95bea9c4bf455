#!/bin/bash
# CPSAM batch 1: split-K 4 for the <=192-tile weight gradients at m = 1024 (A/B by env)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s29
mkdir -p $O
for v in 4096 1024 4096 1024; do
  BE_WGRAD_SPLIT_MIN_M=$v timeout -k 10 200 python tools/cpsam_train_bench.py --batch 1 --steps 30 > $O/train_$v.jsonl 2>&1 || { tail $O/train_$v.jsonl; exit 1; }
  echo min_m=$v $(grep bench $O/train_$v.jsonl | cut -c1-140)
done
echo done
