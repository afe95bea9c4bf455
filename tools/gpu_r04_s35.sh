#!/bin/bash
# round 4 step 35: CM = 64 fused pairs with each chunk's actA affine loaded before the barrier ahead of
# its halo commit (BE_PAIR_EARLY_AFF=1, on top of the LATE default): numerics, phase profile, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s35
mkdir -p $O
BE_PAIR_EARLY_AFF=1 timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/test_early.log 2>&1 || { tail -30 $O/test_early.log; exit 1; }
tail -1 $O/test_early.log
for l in 0 1; do
  BE_PAIR_EARLY_AFF=$l timeout -k 10 200 python3 tools/pair_phase_profile.py > $O/phases_early$l.jsonl 2> $O/phases_early$l.err || { tail -20 $O/phases_early$l.err; exit 1; }
done
python3 - <<PY
import json
for l in (0, 1):
    for line in open("$O/phases_early%d.jsonl" % l):
        d = json.loads(line)
        if d["cm"] == 64:
            c = d["cycles_per_tile"]; print("early", l, d["cin"], d["inmode"], c["halo_commit"], sum(c.values()))
PY
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'))")" | tee -a $O/summary.txt
}
run early0_a BE_PAIR_EARLY_AFF=0
run early1_a BE_PAIR_EARLY_AFF=1
run early0_b BE_PAIR_EARLY_AFF=0
run early1_b BE_PAIR_EARLY_AFF=1
