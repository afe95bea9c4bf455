#!/bin/bash
# full GPU suite + smoke + full 1-GPU bench on the current tree
set -o pipefail
R=$PWD
O=$R/gpurun_out/s25
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log
echo done
