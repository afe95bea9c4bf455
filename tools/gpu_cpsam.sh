#!/bin/bash
# CPSAM training: GPU numerics tests, then the fine-tune step bench (engine vs autograd).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpsam_train_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/cpsam_gpu_tests.log 2>&1
rc=$?; tail -12 gpurun_out/cpsam_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/cpsam_train_bench.py --batch 1 8 --steps 10 ${CPSAM_BENCH_ARGS:-} > gpurun_out/cpsam_bench.log 2>&1
rc=$?; tail -8 gpurun_out/cpsam_bench.log; exit $rc
