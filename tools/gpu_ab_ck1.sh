#!/bin/bash
# A/B of the 1x1-conv chunk width: numerics tests with CK1=64, then per-layer times for 32 and 64.
set -o pipefail
mkdir -p gpurun_out/ab_ck1
BE_CONV_CK1=64 timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_ck1/tests.log 2>&1 || exit $?
for v in 32 64; do
  BE_CONV_CK1=$v timeout -k 10 300 python3 tools/conv_roofline.py --mode time > gpurun_out/ab_ck1/time_$v.jsonl 2> gpurun_out/ab_ck1/time_$v.err || exit $?
done
BE_CONV_CK1=64 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-extras --no-served > gpurun_out/ab_ck1/bench64.log 2>&1
