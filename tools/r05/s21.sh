#!/bin/bash
# round 5 step 21: headline A/Bs: the 56^2 level on the implicit-GEMM conv (BE_CPNET_IGEMM_LEVELS=2,3),
# the pair-kernel grid (CUs left to the mask stream) and the mask-stream priority with the
# ping-pong kernels; mask-stage census
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s21
mkdir -p $O
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u tools/headline_ab.py > $O/$name.json 2>>$O/head_ab.err || exit 1
  echo "$name $(cut -c1-110 $O/$name.json)" | tee -a $O/summary.txt
}
for r in 1 2; do
  run base_$r BE_CPNET_IGEMM_LEVELS=3
  run ig23_$r BE_CPNET_IGEMM_LEVELS=2,3
  run grid240_$r BE_PAIR_GRID=240
  run prio_$r BE_MASK_STREAM_PRIO=-1
done
timeout -k 10 200 python -u tools/mask_census.py > $O/mask_census.json 2>$O/mask_census.err || { tail $O/mask_census.err; exit 1; }
cat $O/mask_census.json | cut -c1-1500
