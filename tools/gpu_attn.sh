#!/bin/bash
# Attention kernels at the CPSAM fine-tune shape: event timing, kernel-trace stats, one SQ counter pass.
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/attn
timeout -k 10 120 python3 tools/attn_bench.py > $R/gpurun_out/attn/time.jsonl 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --bias 0 >> $R/gpurun_out/attn/time.jsonl 2>&1 || exit $?
cat $R/gpurun_out/attn/time.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/attn/prof -o attn -- python3 $R/tools/attn_bench.py --iters 5 > $R/gpurun_out/attn/prof.log 2>&1 || exit $?
if [ -n "$PMC" ]; then
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $R/gpurun_out/attn/pmc -o sq -- python3 $R/tools/attn_bench.py --iters 2 > $R/gpurun_out/attn/pmc.log 2>&1 || exit $?
fi
find $R/gpurun_out/attn -name "*.csv" | head
