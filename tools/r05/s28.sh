#!/bin/bash
# round 5 step 28: batch-1 latency anatomy (kernel trace of tools/latency_b1.py, device and host
# input) + the cellpose tests on the current build (label lookup run-lengths, percentile runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s28
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 200 python3 tools/latency_b1.py --iters 30 > $O/b1_plain.json 2>&1 || { tail $O/b1_plain.json; exit 1; }
cat $O/b1_plain.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o t -- python3 $R/tools/latency_b1.py --iters 12 > $O/b1_trace.log 2>&1 || { tail $O/b1_trace.log; exit 1; }
cd $R && python3 tools/b1_timeline.py $O/b1/t_kernel_trace.csv --iters 3 > $O/b1_timeline.txt 2>&1; cat $O/b1_timeline.txt | head -70
