#!/bin/bash
# round 5 step 38: GPU component-size filter (EM remove_small): EM tests + volume bench; then the
# s37 re-check A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s38
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_em_watershed.py tests/test_em_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 400 python3 -u tools/em_volume_bench.py --z 256 --split-touching > $O/em_volume.json 2> $O/em_volume.err || { tail -20 $O/em_volume.err; exit 1; }
grep metric $O/em_volume.json | cut -c1-700
bash tools/r05/s37.sh || exit 1
