#!/bin/bash
# round 5 step 32: DPP horizontal neighbours in the diffusion queue (3 LDS reads per pixel instead
# of 9): tests, mask-stage + headline + batch-1 A/B against the all-LDS build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s32
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
for r in 1 2; do
  for cfg in dpp nodpp; do
    E=""; [ $cfg = nodpp ] && E="BE_HIP_LIB=$VD/nodpp/libbe_hip.so"
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
for cfg in dpp nodpp; do
  E=""; [ $cfg = nodpp ] && E="BE_HIP_LIB=$VD/nodpp/libbe_hip.so"
  env $E timeout -k 10 200 python3 -u tools/mask_bench.py --variants base --reps 5 > $O/mask_$cfg.jsonl 2>> $O/mask.err || exit 1
  echo "mask $cfg $(cut -c1-90 $O/mask_$cfg.jsonl)"
  env $E timeout -k 10 200 python3 tools/latency_b1.py --iters 30 > $O/b1_$cfg.json 2>/dev/null || exit 1
  echo "b1 $cfg $(cat $O/b1_$cfg.json)"
done
