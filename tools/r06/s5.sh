#!/bin/bash
# round 6, s5: 3-D EM tile-shape sweep, part 2, then the kernel table of one config
set -o pipefail
mkdir -p gpurun_out/r06/s5
cd /root/repo
timeout -k 10 500 python -u tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4,64:256:8,128:256:2,128:256:4,64:384:4,96:384:2 > gpurun_out/r06/s5/sweep.jsonl 2>&1 || { tail -20 gpurun_out/r06/s5/sweep.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06/s5/sweep.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]
        print(c["tile"], c["tiles_per_call"], round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s", c["stage_timings_s_rank0"]["inference"], c["stage_timings_s_rank0"]["label"], d["max_memory_allocated_gb"])
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r06/s5/prof -o em3d -- python3 /root/repo/tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > /root/repo/gpurun_out/r06/s5/prof.log 2>&1 || { tail -20 /root/repo/gpurun_out/r06/s5/prof.log; exit 1; }
find /root/repo/gpurun_out/r06/s5/prof -name "*kernel_stats.csv" | head -3
