#!/bin/bash
# round 4 step 37: CM = 64 fused pairs (no skip operand) with the stage-A epilogue's actB affine loaded
# before its barrier (BE_PAIR_EPIA=1, on top of LATE + ROLL + EARLY): numerics, phase profile, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s37
mkdir -p $O
BE_PAIR_EPIA=1 timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/test_epia.log 2>&1 || { tail -30 $O/test_epia.log; exit 1; }
tail -1 $O/test_epia.log
for l in 0 1; do
  BE_PAIR_EPIA=$l timeout -k 10 200 python3 tools/pair_phase_profile.py > $O/phases_epia$l.jsonl 2> $O/phases_epia$l.err || { tail -20 $O/phases_epia$l.err; exit 1; }
done
python3 - <<PY
import json
for l in (0, 1):
    for line in open("$O/phases_epia%d.jsonl" % l):
        d = json.loads(line)
        if d["cm"] == 64:
            c = d["cycles_per_tile"]; print("epia", l, d["cin"], d["inmode"], c["stageA_epi"], sum(c.values()))
PY
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'))")" | tee -a $O/summary.txt
}
run epia0_a BE_PAIR_EPIA=0
run epia1_a BE_PAIR_EPIA=1
run epia0_b BE_PAIR_EPIA=0
run epia1_b BE_PAIR_EPIA=1
