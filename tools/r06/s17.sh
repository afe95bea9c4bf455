#!/bin/bash
# round 6, s17: native EM label counts (test), then the N > 1 rehearsal again (s6)
set -o pipefail
mkdir -p gpurun_out/r06/s17
cd /root/repo
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_em_watershed.py -m gpu > gpurun_out/r06/s17/tests.log 2>&1 || { tail -30 gpurun_out/r06/s17/tests.log; exit 1; }
tail -2 gpurun_out/r06/s17/tests.log
bash tools/r06/s6.sh
