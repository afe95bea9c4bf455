#!/bin/bash
# round 5 step 29: mask kernels that fit beside a pair-kernel workgroup (LDS <= ~32 KiB): the
# 256-thread diffusion queue (default) vs the 512-thread build, and 16-pixel follow-flows tiles at
# every batch vs the size-based choice; headline A/B, two alternating rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s29
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
for r in 1 2; do
  for cfg in base dq512 ft16; do
    case $cfg in
      base) E="";;
      dq512) E="BE_HIP_LIB=$VD/dq512/libbe_hip.so";;
      ft16) E="BE_FOLLOW_TILE=16";;
    esac
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
for cfg in base dq512 ft16; do
  case $cfg in
    base) E="";;
    dq512) E="BE_HIP_LIB=$VD/dq512/libbe_hip.so";;
    ft16) E="BE_FOLLOW_TILE=16";;
  esac
  env $E timeout -k 10 200 python3 -u tools/mask_bench.py --variants base --reps 5 > $O/mask_$cfg.jsonl 2>> $O/mask.err || exit 1
  echo "mask $cfg $(cut -c1-90 $O/mask_$cfg.jsonl)"
done
