#!/bin/bash
# round 5 step 5: headline A/B (graphed network stage on / off, alternating processes) + Cellpose GPU
# tests; then one PMC pass over the macro-tile GEMM vs hipBLASLt on the batch-8 forward shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$PWD
O=$R/gpurun_out/r05/s5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cellpose_gpu.py tests/test_cpnet_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for gmax in 64 0; do
    BE_CELLPOSE_GRAPH_MAX_B=$gmax timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>>$O/head_ab.err || exit 1
  done
done
cut -c1-220 $O/head_ab.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d $O/pmc -o p -- python3 $R/tools/gemm_mt_bench.py --batches 8 --only "fwd b8" --rounds 2 --reps 5 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $O/pmc/p_counter_collection.csv --top 14 > $O/pmc_summary.txt || exit 1
rm -f $O/pmc/p_counter_collection.csv $O/pmc/p_kernel_trace.csv
grep -E "^void|^Cijk|MFMA_BUSY|WAIT_ANY|conflicts" $O/pmc_summary.txt | cut -c1-150 | head -60
