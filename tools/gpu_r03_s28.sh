#!/bin/bash
# CPSAM: split-K 2 / 4 for the 4096-wide fp32 weight gradients (A/B by env)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s28
mkdir -p $O
for v in 0 2 4 0 2; do
  BE_WGRAD_SPLIT_WIDE=$v timeout -k 10 200 python tools/cpsam_train_bench.py --batch 8 --steps 20 > $O/train_$v.jsonl 2>&1 || { tail $O/train_$v.jsonl; exit 1; }
  echo split=$v $(grep bench $O/train_$v.jsonl | cut -c1-140)
done
echo done
