#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/train_bench.py --batch 8 32 --phases > gpurun_out/train_bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_bench.py --batch 8 32 --norm group >> gpurun_out/train_bench.log 2>&1 || exit $?
mkdir -p gpurun_out/tprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof -o train -- python3 tools/train_bench.py --batch 8 --steps 5 > gpurun_out/tprof/stdout.log 2>&1
echo "prof rc=$?" >> gpurun_out/tprof/stdout.log
