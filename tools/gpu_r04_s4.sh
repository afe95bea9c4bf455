#!/bin/bash
# round 4 step 4: PMC passes over the igemm conv (L3, bn65, plain) and the bf16 GEMM (fwd qkv, B=8)
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r04/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for pass in 1 2; do
  if [ $pass = 1 ]; then PMC=$P1; else PMC=$P2; fi
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/conv_p$pass -o p -- \
    python3 $R/tools/igemm_bench.py --only L3 --bns 65 --variants plain --no-ref --reps 3 > $R/gpurun_out/r04/pmc/conv_p$pass.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/conv_p$pass.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/gemm_p$pass -o p -- \
    python3 $R/tools/gemm_bf16_bench.py --only "fwd qkv" --impls hip,torch --batches 8 --reps 3 > $R/gpurun_out/r04/pmc/gemm_p$pass.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/gemm_p$pass.log; exit 1; }
done
ls -R $R/gpurun_out/r04/pmc | head -30
