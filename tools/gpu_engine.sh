#!/bin/bash
# Training-engine GPU session: kernel/engine numerics, then the fine-tune step bench (hip vs autograd).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpnet_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/engine_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python tools/engine_check.py 2 64 > gpurun_out/engine_check.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_bench.py --batch 8 32 --engine hip --phases > gpurun_out/engine_bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_bench.py --batch 8 --engine autograd >> gpurun_out/engine_bench.log 2>&1
