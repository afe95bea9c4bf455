#!/bin/bash
# MX scale-lane probe; then conv co-major A/B and CPSAM rowcol block counts (from s8)
set -o pipefail
O=$PWD/gpurun_out/s9
mkdir -p $O
for v in main k1; do
  L=$PWD/bioengine_worker_amd/_native/libbe_hip.so; [ $v = k1 ] && L=$PWD/bioengine_worker_amd/_native/variants/k1/libbe_hip.so
  BE_HIP_LIB=$L timeout -k 10 120 python3 tools/mx_scale_probe.py > $O/mx_probe_$v.json 2> $O/mx_probe_$v.err || { tail $O/mx_probe_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/mx_probe_$v.json'))
for m in ('0','1','5'):
    print('$v', m, [(g['k'][0], g['exp'], g['same_row_blocks']) for g in d['rows'][m]])
"
done
timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_main.jsonl 2> $O/all_main.err || { tail $O/all_main.err; exit 1; }
BE_HIP_LIB=$PWD/bioengine_worker_amd/_native/variants/comaj/libbe_hip.so timeout -k 10 200 python3 tools/conv_deep_ab.py --all --nw 0 > $O/all_comaj.jsonl 2> $O/all_comaj.err || { tail $O/all_comaj.err; exit 1; }
tail -1 $O/all_main.jsonl; tail -1 $O/all_comaj.jsonl
for nb in 512 1024 2048; do
  BE_ROWCOL_BLOCKS=$nb timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 --steps 30 > $O/cpsam_rb$nb.jsonl 2>&1 || { tail $O/cpsam_rb$nb.jsonl; exit 1; }
  echo "blocks $nb $(grep bench $O/cpsam_rb$nb.jsonl | cut -c1-120)"
done
echo done
# cross-batch net/mask overlap: 64 images as two 32-image micro-batches on two streams vs 32 per step
timeout -k 10 300 python3 bench.py --no-extras --no-served --batch 64 --chunks 2 --steps 10 --warmup 3 > $O/bench_b64c2.json 2> $O/bench_b64c2.err || { tail $O/bench_b64c2.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-extras --no-served --batch 32 --steps 20 --warmup 5 > $O/bench_b32.json 2> $O/bench_b32.err || { tail $O/bench_b32.err; exit 1; }
cut -c1-200 $O/bench_b64c2.json $O/bench_b32.json
echo done3
