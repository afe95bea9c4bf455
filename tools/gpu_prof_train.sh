#!/bin/bash
# rocprofv3 kernel stats of the fine-tune step (hip engine), batch 8 x 256^2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/tprof_eng
timeout -k 10 300 python -u -m pytest tests/test_cpnet_engine_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/engine_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof_eng -o train -- python3 tools/train_bench.py --batch 8 --steps 5 --engine hip > gpurun_out/tprof_eng/stdout.log 2>&1
echo "prof rc=$?" >> gpurun_out/tprof_eng/stdout.log
