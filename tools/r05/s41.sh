#!/bin/bash
# round 5 step 41: LDS-hash component counts (BE_COMP_KEEP=1) vs the torch.unique sort: EM tests +
# volume bench A/B, two rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s41
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_em_watershed.py tests/test_em_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
for r in 1 2; do
  for ck in 1 0; do
    BE_COMP_KEEP=$ck timeout -k 10 400 python3 -u tools/em_volume_bench.py --z 256 --split-touching > $O/em_volume_ck${ck}_$r.json 2> $O/em_volume_ck${ck}_$r.err || { tail -20 $O/em_volume_ck${ck}_$r.err; exit 1; }
    echo "comp_keep=$ck $(grep -o '"value": [0-9.]*' $O/em_volume_ck${ck}_$r.json) $(grep -o '"remove_small": [0-9.]*' $O/em_volume_ck${ck}_$r.json)"
  done
done
