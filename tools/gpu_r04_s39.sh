#!/bin/bash
# round 4 step 39: the final tree once more (SEPS / EPIA builds added, both off) -- full GPU suite, smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s39
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests_full.log 2>&1; echo "suite rc=$?"; tail -2 $O/gpu_tests_full.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
