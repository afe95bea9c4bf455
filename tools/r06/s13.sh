#!/bin/bash
# round 6, s13: CPSAM inference GELU-epilogue A/B; kernel table of the 2-D EM line (768/64/16 tiles);
# then the serving bench with the ramp split
set -o pipefail
mkdir -p gpurun_out/r06/s13
cd /root/repo
timeout -k 10 300 python -u tools/cpsam_gelu_ab.py > gpurun_out/r06/s13/cpsam_gelu_ab.jsonl 2>&1 || { tail -20 gpurun_out/r06/s13/cpsam_gelu_ab.jsonl; exit 1; }
grep '^{' gpurun_out/r06/s13/cpsam_gelu_ab.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r06/s13/prof -o em2d -- python3 /root/repo/tools/em2d_bench.py --em-z 64 --sweep 768:64:16 > /root/repo/gpurun_out/r06/s13/prof.log 2>&1 || { tail -20 /root/repo/gpurun_out/r06/s13/prof.log; exit 1; }
find /root/repo/gpurun_out/r06/s13/prof -name "*kernel_stats.csv" | head -3
cd /root/repo
timeout -k 10 300 python -u tools/serve_bench.py --concurrency 1,64 --seconds 4 > gpurun_out/r06/s13/serve.log 2>&1 || { tail -20 gpurun_out/r06/s13/serve.log; exit 1; }
grep '^{' gpurun_out/r06/s13/serve.log | tail -4
