#!/bin/bash
# round 5 step 35: PMC passes (SQ counters only, --kernel-trace, no tracing domains): the level-0
# pair kernels ping-pong (BE_PAIR_PP=1) vs one-group (=0), and the round-5 mask-stage kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/s35
mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
cd /tmp && export TMPDIR=/tmp
for pp in 1 0; do
  BE_PAIR_PP=$pp BE_PAIR_PP_STEM=$pp timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pairs_pp$pp -o p -- python3 $R/tools/pair_bench.py --only-pairs --reps 2 > $O/pairs_pp$pp.log 2>&1 || { tail $O/pairs_pp$pp.log; exit 1; }
done
timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/masks -o p -- python3 $R/tools/mask_bench.py --variants base --reps 2 > $O/masks.log 2>&1 || { tail $O/masks.log; exit 1; }
cd $R
for d in pairs_pp1 pairs_pp0; do python3 tools/pmc_summary.py $O/$d/p_counter_collection.csv --match conv_pair --top 8 > $O/${d}_summary.txt || exit 1; done
python3 tools/pmc_summary.py $O/masks/p_counter_collection.csv --top 10 > $O/masks_summary.txt || exit 1
head -60 $O/pairs_pp1_summary.txt
rm -rf $O/pairs_pp1 $O/pairs_pp0 $O/masks
