#!/bin/bash
# c=1 latency by layer on one box: direct runner.eval, router->replica (handle), full hub path.
set -o pipefail
mkdir -p gpurun_out/c1l
timeout -k 10 200 python tools/latency_b1.py --host > gpurun_out/c1l/latency.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 5 --layer handle > gpurun_out/c1l/handle.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 5 --layer hub > gpurun_out/c1l/hub.log 2>&1 || exit $?
BIOENGINE_REPLICA_MODE=local timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 5 --layer handle --replica-mode local > gpurun_out/c1l/local_handle.log 2>&1
