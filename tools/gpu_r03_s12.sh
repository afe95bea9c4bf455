#!/bin/bash
set -o pipefail
O=$PWD/gpurun_out/s12
mkdir -p $O
timeout -k 10 200 python3 tools/debug_stream.py > $O/debug.log 2>&1 || { tail -20 $O/debug.log; exit 1; }
cat $O/debug.log | grep -v amdgpu.ids
