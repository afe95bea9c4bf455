#!/bin/bash
# round 6, s7: level-1 half-blocks on the 12 x 16 geometry (two workgroups per CU): oracle tests,
# per-call A/B, headline A/B (alternating arms)
set -o pipefail
mkdir -p gpurun_out/r06/s7
cd /root/repo
BE_PAIR_G12=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pair.py -m gpu > gpurun_out/r06/s7/test_g12.log 2>&1 || { tail -30 gpurun_out/r06/s7/test_g12.log; exit 1; }
tail -1 gpurun_out/r06/s7/test_g12.log
for g in 0 1; do
  BE_PAIR_G12=$g timeout -k 10 200 python -u tools/pair_bench.py --only-pairs > gpurun_out/r06/s7/pairs_g12_$g.jsonl 2>&1 || exit 1
  echo "G12=$g"; grep '"pair"' gpurun_out/r06/s7/pairs_g12_$g.jsonl | python -c "import sys,json; [print(d['pair'], d['ms']) for d in map(json.loads, sys.stdin)]"
done
for r in 1 2; do for g in 0 1; do
  BE_PAIR_G12=$g timeout -k 10 200 python -u tools/headline_ab.py > gpurun_out/r06/s7/headline_g12_${g}_r$r.json 2>&1 || exit 1
  echo "G12=$g r$r $(grep imgs_per_s gpurun_out/r06/s7/headline_g12_${g}_r$r.json | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['imgs_per_s'], d.get('imgs_per_sec_sequential_batches'), d['p50_ms_b1'])")"
done; done
