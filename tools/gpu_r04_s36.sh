#!/bin/bash
# round 4 step 36: final tree with the level-1 pair builds on by default -- full GPU suite, smoke,
# default 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s36
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests_full.log 2>&1; echo "suite rc=$?"; tail -2 $O/gpu_tests_full.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
# then the EPIA A/B of tools/gpu_r04_s37.sh
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
