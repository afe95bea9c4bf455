#!/bin/bash
# round 5 step 37: re-check the s21 arms with the round-5 mask stage: 56^2 on the implicit-GEMM
# conv (BE_CPNET_IGEMM_LEVELS=2,3) and 240 pair-kernel workgroups; two alternating rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s37
mkdir -p $O
for r in 1 2; do
  for cfg in base ig23 grid240; do
    case $cfg in
      base) E="";;
      ig23) E="BE_CPNET_IGEMM_LEVELS=2,3";;
      grid240) E="BE_PAIR_GRID=240";;
    esac
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
