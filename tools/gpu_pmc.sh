#!/bin/bash
# PMC counters of the conv layers (own run: --pmc with --kernel-trace only).  Output: gpurun_out/pmc
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc -o conv -- python3 tools/conv_pmc.py > gpurun_out/pmc/stdout.log 2>&1
rc=$?
echo "pmc rc=$rc" >> gpurun_out/pmc/stdout.log
exit $rc
