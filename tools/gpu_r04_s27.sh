#!/bin/bash
# round 4 step 27: IVF full-probe failure -- recall through VectorIndex.search as is / synced, and
# with the all-lists probe fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s27
mkdir -p $O
timeout -k 10 200 python3 tools/ivf_lifetime_check.py > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
cat $O/check.log
timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_search_gpu.py > $O/search_test.log 2>&1; echo "search test rc=$?"; tail -3 $O/search_test.log
