#!/bin/bash
# round 5 step 31: defaults after s29 (512-thread diffusion queue, 16-pixel follow tiles): cellpose
# tests, headline A/B vs 32-pixel follow tiles, mask-stage time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s31
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
for r in 1 2; do
  for cfg in base ft32; do
    case $cfg in
      base) E="";;
      ft32) E="BE_FOLLOW_TILE=32";;
    esac
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
for cfg in base ft32; do
  case $cfg in
    base) E="";;
    ft32) E="BE_FOLLOW_TILE=32";;
  esac
  env $E timeout -k 10 200 python3 -u tools/mask_bench.py --variants base --reps 5 > $O/mask_$cfg.jsonl 2>> $O/mask.err || exit 1
  echo "mask $cfg $(cut -c1-90 $O/mask_$cfg.jsonl)"
done
timeout -k 10 200 python3 tools/latency_b1.py --iters 30 > $O/b1_plain.json 2>&1 || exit 1
cat $O/b1_plain.json
