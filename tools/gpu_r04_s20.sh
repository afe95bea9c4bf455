#!/bin/bash
# round 4 step 20: headline pipeline A/B -- mask-recovery stream priority and the fused-pair grid
# (CUs left free for the mask kernels that run beside the next batch's network)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s20
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'))")" | tee -a $O/summary.txt
}
run base0 BE_X=0
run prio BE_MASK_STREAM_PRIO=-1
run grid240 BE_PAIR_GRID=240
run grid224 BE_PAIR_GRID=224
run prio_grid240 BE_MASK_STREAM_PRIO=-1 BE_PAIR_GRID=240
run base1 BE_X=1
