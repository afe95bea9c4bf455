#!/bin/bash
# round 4 step 5: full bench.py (headline + extras incl. the new EM-volume / model-runner lines,
# batched search serving, CPSAM with per-shape GEMM choice)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u bench.py > gpurun_out/r04/s5_bench.log 2>&1; rc=$?
tail -c 6000 gpurun_out/r04/s5_bench.log
exit $rc
