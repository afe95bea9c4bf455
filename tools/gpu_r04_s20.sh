#!/bin/bash
# round 4 step 20: (1) process-replica hop on the box's CPU: parallel ring copies, malloc tuning;
# (2) served Cellpose c=1 with the old / new copy path; (3) headline pipeline A/B -- mask-recovery
# stream priority and the fused-pair grid (CUs left free for the mask kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r04/s20
mkdir -p $O
for cfg in "1 0" "4 0" "1 1" "4 1"; do
  set -- $cfg
  BE_RING_COPY_THREADS=$1 BE_REPLICA_MALLOC=$2 timeout -k 10 120 python3 tools/replica_hop_bench.py --reps 400 >> $O/hop.jsonl 2>> $O/hop.err || { tail $O/hop.err; exit 1; }
done
for cfg in "1 0" "4 1" "1 0" "4 1"; do
  set -- $cfg
  BE_RING_COPY_THREADS=$1 BE_REPLICA_MALLOC=$2 timeout -k 10 240 python3 tools/serve_bench.py --concurrency 1 --seconds 5 > $O/serve_c1_t$1_m$2.log 2>&1 || { tail $O/serve_c1_t$1_m$2.log; exit 1; }
  echo "serve c1 threads=$1 malloc=$2 $(grep '"concurrency"' $O/serve_c1_t$1_m$2.log)" | tee -a $O/summary.txt
done
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'))")" | tee -a $O/summary.txt
}
run base0 BE_X=0
run prio BE_MASK_STREAM_PRIO=-1
run grid240 BE_PAIR_GRID=240
run prio_grid240 BE_MASK_STREAM_PRIO=-1 BE_PAIR_GRID=240
run base1 BE_X=1
