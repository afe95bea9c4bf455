#!/bin/bash
# round 6, s20: watershed sweep knobs on the 3-D line's post-processing (64 x 2048^2 slab)
set -o pipefail
mkdir -p gpurun_out/r06/s20
cd /root/repo
for arm in 32:4 64:4 16:4 32:8 128:4; do
  ml=${arm%%:*}; ce=${arm##*:}
  BE_WS_MAX_LOCAL=$ml BE_WS_CHECK_EVERY=$ce timeout -k 10 300 python -u tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > gpurun_out/r06/s20/em3d_$ml-$ce.log 2>&1 || { tail -20 gpurun_out/r06/s20/em3d_$ml-$ce.log; exit 1; }
  python - "$ml-$ce" <<'PY'
import json, sys
for l in open(f"gpurun_out/r06/s20/em3d_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]; t = c["stage_timings_s_rank0"]
        print("ws", sys.argv[1], round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s label", t["label"], t.get("split_stages"))
PY
done
