#!/bin/bash
# deep-layer conv options: nw 4 / 8, sched-barrier build
set -o pipefail
O=$PWD/gpurun_out/s6
mkdir -p $O
timeout -k 10 200 python3 tools/conv_deep_ab.py > $O/deep_main.jsonl 2> $O/deep_main.err || { tail $O/deep_main.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/cv_sb/libbe_hip.so timeout -k 10 200 python3 tools/conv_deep_ab.py > $O/deep_sb.jsonl 2> $O/deep_sb.err || { tail $O/deep_sb.err; exit 1; }
cat $O/deep_main.jsonl $O/deep_sb.jsonl | cut -c1-160
echo done
