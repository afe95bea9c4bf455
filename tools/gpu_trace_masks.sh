#!/bin/bash
# Kernel timeline of the mask-recovery stage (one call per variant) for critical-path reading.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/trace_masks
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_masks -o t -- python3 $R/tools/mask_bench.py --variants ${VARIANTS:-dv8} --reps 1 > $R/gpurun_out/trace_masks/stdout.log 2>&1
