#!/bin/bash
# round 4 step 24: the full-probe IVF exact-scan failure of s23 -- the test alone, then a debug of
# the scan kernel's candidate scores; then the rest of the s23 plan (phase profile, suite, bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s24
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_search_gpu.py > $O/search_test.log 2>&1; echo "search test rc=$?"; tail -3 $O/search_test.log
timeout -k 10 200 python3 tools/ivf_scan_debug.py > $O/ivf_debug.log 2>&1 || { tail -20 $O/ivf_debug.log; exit 1; }
cat $O/ivf_debug.log
