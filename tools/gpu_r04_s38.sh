#!/bin/bash
# round 4 step 38: level-0 fused pairs with the output staging in its own LDS region (BE_PAIR_SEPS=1):
# one barrier less per tile; numerics, phase profile, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s38
mkdir -p $O
BE_PAIR_SEPS=1 timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_conv_pair.py > $O/test_seps.log 2>&1 || { tail -30 $O/test_seps.log; exit 1; }
tail -1 $O/test_seps.log
for l in 0 1; do
  BE_PAIR_SEPS=$l timeout -k 10 200 python3 tools/pair_phase_profile.py > $O/phases_seps$l.jsonl 2> $O/phases_seps$l.err || { tail -20 $O/phases_seps$l.err; exit 1; }
done
python3 - <<PY
import json
for l in (0, 1):
    for line in open("$O/phases_seps%d.jsonl" % l):
        d = json.loads(line)
        if d["cm"] == 32:
            c = d["cycles_per_tile"]; print("seps", l, d["cin"], d["inmode"], c["halo_commit"], c["out_epi"], sum(c.values()))
PY
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 bench.py --steps 20 --warmup 3 --no-extras --no-served --no-em > $O/$name.json 2> $O/$name.err || { tail $O/$name.err; exit 1; }
  echo "$name $(python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print(d['value'], d.get('imgs_per_sec_sequential_batches'))")" | tee -a $O/summary.txt
}
run seps0_a BE_PAIR_SEPS=0
run seps1_a BE_PAIR_SEPS=1
run seps0_b BE_PAIR_SEPS=0
run seps1_b BE_PAIR_SEPS=1
