#!/bin/bash
# round 5 step 4: Cellpose GPU tests (graphed network stage), headline A/B graph on/off (alternating
# processes), batch-1 latency
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cellpose_gpu.py tests/test_cpnet_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for gmax in 64 0; do
    BE_CELLPOSE_GRAPH_MAX_B=$gmax timeout -k 10 200 python -u tools/headline_ab.py >> $O/head_ab.jsonl 2>$O/head_ab_$gmax_$r.err || exit 1
  done
done
cut -c1-260 $O/head_ab.jsonl
