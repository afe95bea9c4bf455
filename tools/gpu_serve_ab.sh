#!/bin/bash
# A/B of serving knobs on one box: c=1 latency with and without inline offload, twice each.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    BIOENGINE_BATCH_INLINE=$v timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 4 > gpurun_out/serve_ab_inline${v}_$i.log 2>&1 || exit $?
    echo "inline=$v run=$i $(grep concurrency gpurun_out/serve_ab_inline${v}_$i.log)"
  done
done
