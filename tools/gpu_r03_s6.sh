#!/bin/bash
# fused output head (conv_pair_head): GPU tests + headline bench; deep-layer conv options (nw 4 / 8,
# sched-barrier build)
set -o pipefail
O=$PWD/gpurun_out/s6
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_pair.py tests/test_cpnet_engine_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 bench.py --no-extras --no-served --steps 20 --warmup 5 > $O/bench_head.json 2> $O/bench_head.err || { tail $O/bench_head.err; exit 1; }
BE_CPNET_HEAD=0 timeout -k 10 300 python3 bench.py --no-extras --no-served --steps 20 --warmup 5 > $O/bench_nohead.json 2> $O/bench_nohead.err || { tail $O/bench_nohead.err; exit 1; }
cut -c1-200 $O/bench_head.json $O/bench_nohead.json
timeout -k 10 200 python3 tools/conv_deep_ab.py > $O/deep_main.jsonl 2> $O/deep_main.err || { tail $O/deep_main.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/cv_sb/libbe_hip.so timeout -k 10 200 python3 tools/conv_deep_ab.py > $O/deep_sb.jsonl 2> $O/deep_sb.err || { tail $O/deep_sb.err; exit 1; }
cat $O/deep_main.jsonl $O/deep_sb.jsonl | cut -c1-160
echo done
