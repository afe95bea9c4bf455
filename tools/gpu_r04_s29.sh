#!/bin/bash
# round 4 step 29: is test_cross_batch_stream_and_locked_eval_match_eval (failed once in s28, after
# the native-pointer lifetime change) deterministic?  Two runs of it, then the whole GPU suite
# without -x (every failure listed), then the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s29
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py -k cross_batch > $O/xbatch_$i.log 2>&1; echo "cross_batch run $i rc=$?"; tail -1 $O/xbatch_$i.log
done
BE_NATIVE_PTR_KEEP=0 timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py -k cross_batch > $O/xbatch_nokeep.log 2>&1; echo "cross_batch (bare pointers) rc=$?"; tail -1 $O/xbatch_nokeep.log
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tests_full.log 2>&1; echo "suite rc=$?"; tail -4 $O/gpu_tests_full.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 1500 $O/bench_default.json
