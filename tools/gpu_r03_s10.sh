#!/bin/bash
# fp8 fragments in the instruction's K order (FP8_KLAYOUT=1): fp8 tests incl. the MX path, ViT bench;
# CPSAM + GELU-kernel tests (branch-free erf)
set -o pipefail
O=$PWD/gpurun_out/s10
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8.py tests/test_cpsam_train_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 tools/fp8_bench.py > $O/fp8_bench.jsonl 2> $O/fp8_bench.err || { tail $O/fp8_bench.err; exit 1; }
cat $O/fp8_bench.jsonl | cut -c1-300
echo done
