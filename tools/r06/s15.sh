#!/bin/bash
# round 6, s15: the whole GPU test suite on the final tree, then the N > 1 rehearsal of bench.py (s6)
set -o pipefail
mkdir -p gpurun_out/r06/s15
cd /root/repo
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/s15/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r06/s15/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/r06/s6.sh
