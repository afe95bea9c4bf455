#!/bin/bash
# round 6, s2: gemm_8p persistent (grid 256) vs one block per tile; K sweep
set -o pipefail
mkdir -p gpurun_out/r06/s2
cd /root/repo
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_8p.py > gpurun_out/r06/s2/test.log 2>&1 || { tail -30 gpurun_out/r06/s2/test.log; exit 1; }
tail -1 gpurun_out/r06/s2/test.log
SH=8192x3072x1024,8192x4096x1024,8192x1024x4096,8192x1024x1024,4096x4096x1024,4096x4096x4096,1024x4096x1024
timeout -k 10 300 python -u tools/gemm_8p_bench.py --rounds 5 --shapes $SH > gpurun_out/r06/s2/pers.jsonl 2>&1 || exit 1
BE_GEMM_8P_GRID=0 timeout -k 10 300 python -u tools/gemm_8p_bench.py --rounds 5 --shapes $SH > gpurun_out/r06/s2/perblock.jsonl 2>&1 || exit 1
echo persistent; grep '"impl"' gpurun_out/r06/s2/pers.jsonl
echo per-block; grep '"impl": "8p"' gpurun_out/r06/s2/perblock.jsonl
