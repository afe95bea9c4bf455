#!/bin/bash
# round 5 step 40: EM labelling A/B (s39) + the full GPU suite + the default bench on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s40
mkdir -p $O
stop() { [ "$1" -ge 124 ] && { echo "stopping after rc=$1"; exit "$1"; }; return 0; }
bash tools/r05/s39.sh; rc=$?; echo "s39 rc=$rc"; stop $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -4 $O/gpu_tests.log; stop $rc
timeout -k 10 900 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log; tail -c 600 $O/bench.log
exit $rc
