#!/bin/bash
# round 5 step 47: kernel table of the headline step on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/s47
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/head -o t -- python3 $R/bench.py --no-extras --no-served --no-em --steps 5 --warmup 2 > $O/head.log 2>&1 || { tail $O/head.log; exit 1; }
cd $R && python3 tools/kt_steps.py $O/head/t_kernel_trace.csv --steps 4 --marker "tiles_gather_kernel" --top 45 --width 120 > $O/kt_step_headline_b32_final.txt || exit 1
head -40 $O/kt_step_headline_b32_final.txt
rm -rf $O/head
