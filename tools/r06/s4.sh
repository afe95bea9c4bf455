#!/bin/bash
# round 6, s4: 3-D EM tile-shape sweep (64 x 2048^2 slab), then a kernel profile of the default
set -o pipefail
mkdir -p gpurun_out/r06/s4
cd /root/repo
timeout -k 10 500 python -u tools/em3d_bench.py --em3d-z 64 --sweep 32:128:4,32:128:16,32:256:4,64:256:2,64:256:4,48:192:8 > gpurun_out/r06/s4/sweep.jsonl 2>&1 || { tail -20 gpurun_out/r06/s4/sweep.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06/s4/sweep.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]
        print(c["tile"], c["tiles_per_call"], round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s", c["stage_timings_s_rank0"]["inference"], d["max_memory_allocated_gb"])
PY
