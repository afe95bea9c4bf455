#!/bin/bash
# round 4 step 9: whole-network A/B with the ping-pong deep convs, served-path overhead split,
# served search with the native thumbnail encoder, PMC of the ping-pong kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u tools/cpnet_engine_ab.py --reps 10 --configs perlayer_deep,pp_deep,pp_deep_cfg1,pp_deep_L1 > gpurun_out/r04/s9_engine.jsonl 2>&1 || { tail -20 gpurun_out/r04/s9_engine.jsonl; exit 1; }
grep '^{' gpurun_out/r04/s9_engine.jsonl
timeout -k 10 300 python -u tools/search_serve_bench.py --concurrency 1,64 --seconds 4 > gpurun_out/r04/s9_search.log 2>&1 || { tail -20 gpurun_out/r04/s9_search.log; exit 1; }
grep '^{' gpurun_out/r04/s9_search.log | cut -c1-700
for lay in hub handle; do
  timeout -k 10 200 python -u tools/serve_bench.py --concurrency 1 --seconds 3 --layer $lay > gpurun_out/r04/s9_serve_$lay.log 2>&1 || { tail -20 gpurun_out/r04/s9_serve_$lay.log; exit 1; }
  grep '^{' gpurun_out/r04/s9_serve_$lay.log | cut -c1-400
done
R=$PWD
mkdir -p gpurun_out/r04/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/pp -o p -- \
  python3 $R/tools/pp_bench.py --reps 2 --cfgs 0,2 --only "L3 256->256" --what conv > $R/gpurun_out/r04/pmc/pp.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/pp.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $R/gpurun_out/r04/pmc/ppg -o p -- \
  python3 $R/tools/pp_bench.py --reps 2 --cfgs 0 --only "qkv b8" --what gemm > $R/gpurun_out/r04/pmc/ppg.log 2>&1 || { tail -5 $R/gpurun_out/r04/pmc/ppg.log; exit 1; }
echo pmc done
