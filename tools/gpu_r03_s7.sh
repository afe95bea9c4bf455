#!/bin/bash
# conv: output-channel-major block order (variant comaj) vs shipped, every per-layer conv of the
# headline batch; headline bench with the shipped build.
set -o pipefail
O=$PWD/gpurun_out/s7
mkdir -p $O
timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_main.jsonl 2> $O/all_main.err || { tail $O/all_main.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/comaj/libbe_hip.so timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_comaj.jsonl 2> $O/all_comaj.err || { tail $O/all_comaj.err; exit 1; }
paste -d' ' <(cut -c1-110 $O/all_main.jsonl) <(grep -o '"ms": [0-9.]*' $O/all_comaj.jsonl)
timeout -k 10 300 python3 bench.py --no-extras --no-served --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/comaj/libbe_hip.so timeout -k 10 300 python3 bench.py --no-extras --no-served --steps 20 --warmup 5 > $O/bench_comaj.json 2> $O/bench_comaj.err || { tail $O/bench_comaj.err; exit 1; }
cut -c1-200 $O/bench.json $O/bench_comaj.json

# CPSAM elementwise kernels: rows per block (512 / 1024 / 2048 blocks per launch)
for nb in 512 1024 2048; do
  BE_ROWCOL_BLOCKS=$nb timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 --steps 30 > $O/cpsam_rb$nb.jsonl 2>&1 || { tail $O/cpsam_rb$nb.jsonl; exit 1; }
  echo "blocks $nb $(grep bench $O/cpsam_rb$nb.jsonl | cut -c1-120)"
done
echo done2
