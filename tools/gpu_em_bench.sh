#!/bin/bash
# EM volume bench on one GPU: gather modes (rank0 / sharded) and the 3-D watershed split.
set -o pipefail
mkdir -p gpurun_out/em
Z=${EM_Z:-128}
for g in rank0 sharded; do
  timeout -k 10 300 python tools/em_volume_bench.py --z $Z --gather $g > gpurun_out/em/bench_$g.log 2>&1 || exit $?
done
timeout -k 10 400 python tools/em_volume_bench.py --z ${EM_ZS:-64} --gather rank0 --split-touching > gpurun_out/em/bench_split.log 2>&1
