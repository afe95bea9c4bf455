#!/bin/bash
# c=1 serving anatomy: GPU cellpose/conv tests, batch-1 direct latency, then an untraced served c=1
# run with a cProfile of the replica child (tottime + cumulative).
set -o pipefail
mkdir -p gpurun_out/c1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cellpose_gpu.py tests/test_conv_gpu.py tests/test_style_ops.py tests/test_cpnet_engine_gpu.py > gpurun_out/c1/tests.log 2>&1 || exit $?
timeout -k 10 200 python tools/latency_b1.py --host > gpurun_out/c1/latency.log 2>&1 || exit $?
timeout -k 10 200 python tools/latency_b1.py >> gpurun_out/c1/latency.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1,64 --seconds 5 > gpurun_out/c1/serve.log 2>&1 || exit $?
BE_REPLICA_PROFILE="$PWD/gpurun_out/c1/replica_prof_{pid}.txt" timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 5 > gpurun_out/c1/serve_prof.log 2>&1
