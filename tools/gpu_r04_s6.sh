#!/bin/bash
# round 4 step 6: bf16 GEMM wave-tile configurations (8 waves of 64x64 vs 4 waves of 128x64 / 64x128)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gemm_bf16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/s6_tests.log 2>&1 || { tail -40 gpurun_out/r04/s6_tests.log; exit 1; }
tail -2 gpurun_out/r04/s6_tests.log
timeout -k 10 400 python -u tools/gemm_bf16_bench.py --cfgs 0,1,2,3 --reps 10 > gpurun_out/r04/s6_gemm.jsonl 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r04/s6_gemm.jsonl
timeout -k 10 300 python -u tools/search_serve_bench.py --concurrency 1,64 --seconds 4 > gpurun_out/r04/s6_search.log 2>&1 || { tail -20 gpurun_out/r04/s6_search.log; exit 1; }
grep '^{' gpurun_out/r04/s6_search.log
# PMC over the headline's conv kernels: fused pairs (levels 0/1) and the deep per-layer convs
R=$PWD
mkdir -p gpurun_out/r04/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/pairs -o p -- \
  python3 $R/tools/pair_bench.py --only-pairs --reps 2 > $R/gpurun_out/r04/pmc/pairs.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/pairs.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/deep -o p -- \
  python3 $R/tools/conv_deep_ab.py --reps 2 --nw 0 > $R/gpurun_out/r04/pmc/deep.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/deep.log; exit 1; }
echo pmc done
exit $rc
