#!/bin/bash
# SQ counters of the fp8 GEMM tile configs on the qkv shape (one rocprofv3 pass).
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/fp8pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $R/gpurun_out/fp8pmc -o p -- python3 $R/tools/fp8_pmc.py 16448 2304 768 1,4,6 > $R/gpurun_out/fp8pmc/stdout.log 2>&1
