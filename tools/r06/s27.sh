#!/bin/bash
# round 6, s27: kernel tables of the final EM lines (3-D and 2-D, 64 x 2048^2 slabs)
set -o pipefail
mkdir -p gpurun_out/r06/s27
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r06/s27/prof3d -o em3d -- python3 /root/repo/tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > /root/repo/gpurun_out/r06/s27/prof3d.log 2>&1 || { tail -20 /root/repo/gpurun_out/r06/s27/prof3d.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r06/s27/prof2d -o em2d -- python3 /root/repo/tools/em2d_bench.py --em-z 64 --sweep 768:64:16 > /root/repo/gpurun_out/r06/s27/prof2d.log 2>&1 || { tail -20 /root/repo/gpurun_out/r06/s27/prof2d.log; exit 1; }

cd /root/repo
python3 tools/rocpd_stats.py gpurun_out/r06/s27/prof3d/em3d_results.db --top 30 --start-frac 0.5 > gpurun_out/r06/s27/kt_em3d_final.txt
python3 tools/rocpd_stats.py gpurun_out/r06/s27/prof2d/em2d_results.db --top 30 --start-frac 0.5 > gpurun_out/r06/s27/kt_em2d_final.txt
rm -rf gpurun_out/r06/s27/prof3d gpurun_out/r06/s27/prof2d
head -12 gpurun_out/r06/s27/kt_em3d_final.txt
