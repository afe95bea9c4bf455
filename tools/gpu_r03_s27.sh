#!/bin/bash
# deep 3x3 conv layers: 4 vs 8 waves under the XCD-grouped block order (default now)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s27
mkdir -p $O
timeout -k 10 300 python tools/conv_deep_ab.py --nw 4,8 > $O/deep_nw.jsonl 2>&1 || { tail $O/deep_nw.jsonl; exit 1; }
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/s27/deep_nw.jsonl") if l.startswith("{") and "idx" in l]
by = collections.defaultdict(dict)
for r in rows: by[(r["idx"], r["layer"])][r["nw"]] = r["ms"]
t4 = t8 = tb = 0
for (i, l), d in sorted(by.items()):
    a, b = d.get(4), d.get(8)
    t4 += a or 0; t8 += (b or a or 0); tb += min(x for x in (a, b) if x)
    print(i, l, a, b, "8 wins" if (a and b and b < a * 0.97) else "")
print("total nw4", round(t4, 3), "nw8", round(t8, 3), "best-of", round(tb, 3))
PY
echo done
