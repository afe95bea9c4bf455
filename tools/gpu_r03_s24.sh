#!/bin/bash
# conv2d_nhwc_kernel block order: tile-major (0) vs XCD-grouped co-major (2): numerics, per-layer A/B, headline
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s24
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "conv or cpnet or cellpose or engine" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for o in 0 2; do
  BE_CONV_ORDER=$o timeout -k 10 200 python tools/conv_deep_ab.py --nw 4 > $O/deep_o$o.jsonl 2>&1 || { tail $O/deep_o$o.jsonl; exit 1; }
done
python3 - <<'PY'
import json
for o in (0, 2):
    rows = [json.loads(l) for l in open(f"gpurun_out/s24/deep_o{o}.jsonl") if l.startswith("{")]
    print("order", o, "total ms", round(sum(r.get("ms", 0) for r in rows), 3))
    for r in rows: print("  ", r.get("layer"), r.get("ms"), r.get("TFs"))
PY
for o in 0 2; do
  BE_CONV_ORDER=$o timeout -k 10 200 python bench.py --no-extras --no-served --steps 10 > $O/bench_o$o.log 2>&1 || { tail $O/bench_o$o.log; exit 1; }
  tail -1 $O/bench_o$o.log | cut -c1-260
done
echo done
