#!/bin/bash
# conv_pair grid: one workgroup per CU (0) vs 512 / 1024 smaller tile ranges (load balance next to the
# mask stream of the pipelined headline)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s31
mkdir -p $O
for g in 0 512 1024 0 512 1024; do
  BE_PAIR_GRID=$g timeout -k 10 200 python bench.py --no-extras --no-served --steps 10 > $O/bench_$g.log 2>&1 || { tail $O/bench_$g.log; exit 1; }
  echo grid=$g $(tail -1 $O/bench_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['imgs_per_sec_sequential_batches'])")
done
echo done
