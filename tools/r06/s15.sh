#!/bin/bash
# round 6, s15: the whole GPU test suite on the final tree
set -o pipefail
mkdir -p gpurun_out/r06/s15
cd /root/repo
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/s15/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06/s15/gpu_tests.log
exit $rc
