#!/bin/bash
# round 6, s16: full 1-GPU bench.py (driver defaults) on the final tree
set -o pipefail
mkdir -p gpurun_out/r06/s16
cd /root/repo
timeout -k 10 1000 python -u bench.py > gpurun_out/r06/s16/bench_1gpu.log 2>&1
rc=$?
grep '^{"metric"' gpurun_out/r06/s16/bench_1gpu.log > gpurun_out/r06/s16/bench_1gpu.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06/s16/bench_1gpu.json"))
keys = ["value", "ms_per_step", "imgs_per_sec_sequential_batches", "p50_latency_ms_batch1", "vs_reference_algorithm",
        "served_p50_ms_c1", "served_imgs_per_sec_c64", "served_p50_ms_c64", "served_p99_ms_c64", "served_p99_ms_c64_incl_ramp",
        "vit_embed_imgs_per_s", "finetune_samples_per_sec", "finetune_cpsam_samples_per_sec",
        "finetune_cpsam_batch1_samples_per_sec", "finetune_cpsam_dp_path_ms_b1", "finetune_cpsam_zero_dp_path_ms_b1",
        "cpsam_infer_imgs_per_s", "cpsam_infer_p50_ms_batch1", "em_volume_voxels_per_sec", "em_volume3d_voxels_per_sec"]
for k in keys: print(k, d.get(k))
print("errors", {k: v for k, v in d.items() if k.startswith("extras_error")})
for k in ("em_volume_config", "em_volume3d_config"):
    print(k, d.get(k, {}).get("stage_timings_s_rank0"))
PY
grep -o '"router[^}]*}[^}]*}' gpurun_out/r06/s16/bench_1gpu.log | head -3
exit $rc
