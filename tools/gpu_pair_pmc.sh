#!/bin/bash
# PMC pass over the fused two-conv kernels (tools/pair_bench.py --only-pairs): one rocprofv3 run,
# --pmc with --kernel-trace only (gpurun refuses PMC combined with the tracing domains).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pair_pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT} \
  --kernel-trace --output-format csv -d $R/gpurun_out/pair_pmc/${PASS:-sq} -o p -- python3 $R/tools/pair_bench.py --only-pairs --reps 2 \
  > $R/gpurun_out/pair_pmc/${PASS:-sq}.log 2>&1
