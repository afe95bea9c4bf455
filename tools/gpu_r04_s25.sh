#!/bin/bash
# round 4 step 25: IVF full-probe failure -- GPU vs CPU post-processing of the (correct) scan output
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s25
mkdir -p $O
timeout -k 10 200 python3 tools/ivf_scan_debug.py > $O/ivf_debug.log 2>&1 || { tail -20 $O/ivf_debug.log; exit 1; }
cat $O/ivf_debug.log
