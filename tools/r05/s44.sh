#!/bin/bash
# round 5 step 44: bit-row hole filling with batched row loads: tests, mask stage,
# batch-1 and headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s44
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
timeout -k 10 200 python3 -u tools/mask_bench.py --variants base --reps 5 > $O/mask.jsonl 2> $O/mask.err || { tail $O/mask.err; exit 1; }
cut -c1-120 $O/mask.jsonl
timeout -k 10 200 python3 tools/latency_b1.py --iters 30 > $O/b1.json 2>/dev/null || exit 1
cat $O/b1.json
for r in 1 2; do
  timeout -k 10 200 python -u tools/headline_ab.py > $O/head_$r.json 2>>$O/head_ab.err || exit 1
  echo "head $(cut -c1-100 $O/head_$r.json)"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1k -o t -- python3 $R/tools/latency_b1.py --iters 12 > $O/b1_trace.log 2>&1 || { tail $O/b1_trace.log; exit 1; }
cd $R && python3 tools/b1_timeline.py $O/b1k/t_kernel_trace.csv --iters 2 --gaps 6 > $O/b1_timeline.txt 2>&1; grep -i "iteration\|fill_holes\|diffuse\|follow" $O/b1_timeline.txt | head -12
rm -rf $O/b1k
