#!/bin/bash
# round 6, s10: 2-D EM line tile sweep (64 x 2048^2 slab)
set -o pipefail
mkdir -p gpurun_out/r06/s10
cd /root/repo
timeout -k 10 600 python -u tools/em2d_bench.py --em-z 64 --sweep 512:64:32,512:64:64,768:64:16,1024:64:8,1024:64:16,1024:32:8 > gpurun_out/r06/s10/sweep.jsonl 2>&1 || { tail -20 gpurun_out/r06/s10/sweep.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r06/s10/sweep.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume_config"]; t = c["stage_timings_s_rank0"]
        print(c["tile"], c["overlap"], c["tiles_per_call"], round(d["em_volume_voxels_per_sec"] / 1e6, 1), "Mvox/s", t["inference"], t["label"], t["stats"], d["max_memory_allocated_gb"])
PY
timeout -k 10 300 python -u tools/gemm_infer_ab.py > gpurun_out/r06/s10/gemm_infer_ab.jsonl 2>&1 || { tail -20 gpurun_out/r06/s10/gemm_infer_ab.jsonl; exit 1; }
grep '"impl"' gpurun_out/r06/s10/gemm_infer_ab.jsonl
