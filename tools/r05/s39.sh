#!/bin/bash
# round 5 step 39: EM labelling: wave-combined component counts (vs the torch.unique sort), bit-packed
# closing, 2-D EDT bounded search: tests + volume bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s39
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_em_watershed.py tests/test_em_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
for ck in 1 0; do
  BE_COMP_KEEP=$ck timeout -k 10 400 python3 -u tools/em_volume_bench.py --z 256 --split-touching > $O/em_volume_ck$ck.json 2> $O/em_volume_ck$ck.err || { tail -20 $O/em_volume_ck$ck.err; exit 1; }
  echo "comp_keep_gpu=$ck $(grep metric $O/em_volume_ck$ck.json | cut -c1-80) $(grep -o '"split_stages[^}]*}' $O/em_volume_ck$ck.json)"
done
