#!/bin/bash
# round 4 step 13: served search -- batch-decoded payloads, batch size / concurrent batches A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s13
mkdir -p $O
for cfg in 32:2 16:4 64:2 32:3; do
  b=${cfg%%:*}; c=${cfg##*:}
  BIOENGINE_SEARCH_MAX_BATCH=$b BIOENGINE_SEARCH_CONCURRENT_BATCHES=$c timeout -k 10 240 python -u tools/search_serve_bench.py --concurrency 1,64 --seconds 4 > $O/search_b${b}_c${c}.log 2>&1 || { tail -20 $O/search_b${b}_c${c}.log; exit 1; }
  echo "== batch $b concurrent $c"; grep '^{' $O/search_b${b}_c${c}.log | cut -c1-330
done
