#!/bin/bash
# round 5 step 7: level-0 fused pairs with the epilogue operands issued after the halo commit
# (default) vs the round-4 order (BE_PAIR_TOPEPI=1): numerics, phase profile, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s7
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for l in 1 0; do
  BE_PAIR_TOPEPI=$l timeout -k 10 200 python3 tools/pair_phase_profile.py > $O/phases_top$l.jsonl 2> $O/phases_top$l.err || { tail -20 $O/phases_top$l.err; exit 1; }
done
python3 - <<PY
import json
for l in (1, 0):
    for line in open("$O/phases_top%d.jsonl" % l):
        d = json.loads(line)
        c = d["cycles_per_tile"]; print("top", l, d["cin"], d["cm"], d["inmode"], {k: round(v) for k, v in c.items()}, round(sum(c.values())))
PY
for r in 1 2; do
  for l in 1 0; do
    BE_PAIR_TOPEPI=$l timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
  done
done
cut -c1-200 $O/head_ab.jsonl
