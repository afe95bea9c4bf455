#!/bin/bash
# Sweep of the training-kernel tunables (wgrad reduce chunks, BN block count) + per-kernel microbench.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/train_sweep.jsonl
: > $out
timeout -k 10 120 python tools/train_kernel_bench.py >> $out 2>/dev/null || exit $?
timeout -k 10 120 python tools/train_kernel_bench.py --H 64 --C 128 >> $out 2>/dev/null || exit $?
for bn in 256 1024 2048; do
  BE_BN_BLOCKS=$bn timeout -k 10 120 python tools/train_kernel_bench.py >> $out 2>/dev/null || exit $?
done
for ch in 4 64; do
  BE_WG_CHUNKS=$ch timeout -k 10 120 python tools/train_kernel_bench.py >> $out 2>/dev/null || exit $?
done
for cfg in "BE_BN_BLOCKS=512" "BE_BN_BLOCKS=2048" "BE_WG_CHUNKS=4" "BE_WG_CHUNKS=64"; do
  env $cfg timeout -k 10 120 python tools/train_bench.py --batch 8 --engine hip | sed "s/^/{\"cfg\": \"$cfg\", \"r\": /; s/$/}/" >> $out || exit $?
done
