#!/bin/bash
# PMC pass over the mask-recovery stage (variant 0 only): SQ wait / LDS counters per kernel.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc_masks
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmc_masks -o m -- python3 $R/tools/mask_bench.py --variants 0 --reps 1 > $R/gpurun_out/pmc_masks/stdout.log 2>&1
