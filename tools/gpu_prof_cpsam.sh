#!/bin/bash
# rocprofv3 kernel-trace + stats of the Cellpose-SAM fine-tune step (engine only, batch ${B:-8}).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof_cpsam
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cpsam -o cpsam -- python3 tools/cpsam_train_bench.py --batch ${B:-8} --steps 5 --warmup 2 > gpurun_out/prof_cpsam/stdout.log 2>&1
rc=$?
echo "prof rc=$rc" >> gpurun_out/prof_cpsam/stdout.log
find gpurun_out/prof_cpsam -name "*stats*" >> gpurun_out/prof_cpsam/stdout.log
tail -3 gpurun_out/prof_cpsam/stdout.log
exit $rc
