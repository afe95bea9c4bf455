#!/bin/bash
# Counters of the fp8 GEMM tile configs on the qkv shape, one rocprofv3 pass per call:
#   PASS=sq  (default) SQ wait / MFMA / LDS-conflict counters
#   PASS=mem L2 hit/miss and the TCP->L2 read latency
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/fp8pmc
cd /tmp && export TMPDIR=/tmp
if [ "${PASS:-sq}" = mem ]; then
  CTR="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
else
  CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
fi
timeout -k 10 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $R/gpurun_out/fp8pmc -o ${PASS:-sq} -- python3 $R/tools/fp8_pmc.py ${SHAPE:-16448 2304 768} ${CFGS:-1,4} > $R/gpurun_out/fp8pmc/stdout_${PASS:-sq}.log 2>&1
