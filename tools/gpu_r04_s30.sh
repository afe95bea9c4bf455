#!/bin/bash
# round 4 step 30: follow_flows with 1,024-pixel pooled compaction (full waves) -- identity test
# against the pixel-per-lane launch, the cellpose GPU tests, then the headline A/B (pool 1 vs 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s30
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'), d.get('masks_per_image'))")" | tee -a $O/summary.txt
}
run pool1_a BE_FOLLOW_POOL=1
run pool4_a BE_FOLLOW_POOL=4
run pool1_b BE_FOLLOW_POOL=1
run pool4_b BE_FOLLOW_POOL=4
cd /tmp && export TMPDIR=/tmp
for pl in 1 4; do
  BE_FOLLOW_POOL=$pl timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_pool$pl -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-extras --no-served --no-em > $O/kt_pool$pl.log 2>&1 || { tail $O/kt_pool$pl.log; exit 1; }
done
grep -h "follow_flows" $O/kt_pool*/t_kernel_stats.csv | cut -c1-200
