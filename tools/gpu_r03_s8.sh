#!/bin/bash
# MX-fp8 fc1 -> fc2 (GELU + E8M0-block quantisation in fc1's epilogue), branch-free erf in the GELU
# passes: GPU tests, ViT end-to-end bench; conv co-major A/B; CPSAM rowcol block counts.
set -o pipefail
O=$PWD/gpurun_out/s8
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp8.py tests/test_cpsam_train_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 tools/fp8_bench.py > $O/fp8_bench.jsonl 2> $O/fp8_bench.err || { tail $O/fp8_bench.err; exit 1; }
tail -1 $O/fp8_bench.jsonl
timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_main.jsonl 2> $O/all_main.err || { tail $O/all_main.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/comaj/libbe_hip.so timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_comaj.jsonl 2> $O/all_comaj.err || { tail $O/all_comaj.err; exit 1; }
tail -1 $O/all_main.jsonl; tail -1 $O/all_comaj.jsonl
for nb in 512 1024 2048; do
  BE_ROWCOL_BLOCKS=$nb timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 --steps 30 > $O/cpsam_rb$nb.jsonl 2>&1 || { tail $O/cpsam_rb$nb.jsonl; exit 1; }
  echo "blocks $nb $(grep bench $O/cpsam_rb$nb.jsonl | cut -c1-120)"
done
echo done
