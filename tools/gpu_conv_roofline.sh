#!/bin/bash
# Per-layer conv roofline: timed replay, then three PMC passes (each its own rocprofv3 run,
# --pmc with --kernel-trace only), then the joined markdown table.  rocprofv3 runs end in a
# segfault at process exit AFTER writing their output, so run one pass per call (SKIP_* vars).
set -o pipefail
mkdir -p gpurun_out/roof
R=$PWD
[ -n "$SKIP_TIME" ] || timeout -k 10 300 python3 tools/conv_roofline.py --mode time > gpurun_out/roof/time.jsonl 2> gpurun_out/roof/time.err || exit $?
cd /tmp && export TMPDIR=/tmp
run_pass() {
  timeout -k 10 300 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $R/gpurun_out/roof/$1 -o p -- python3 $R/tools/conv_roofline.py --mode pmc --order $R/gpurun_out/roof/order.json > $R/gpurun_out/roof/$1.log 2>&1
}
[ -n "$SKIP_SQ" ] || run_pass sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU" || exit $?
[ -n "$SKIP_FETCH" ] || run_pass fetch "FETCH_SIZE" || exit $?
[ -n "$SKIP_WRITE" ] || run_pass write "WRITE_SIZE" || exit $?
cd $R
python3 tools/conv_roofline_table.py gpurun_out/roof/time.jsonl gpurun_out/roof/order.json gpurun_out/roof/sq gpurun_out/roof/fetch gpurun_out/roof/write > gpurun_out/roof/table.md
