#!/bin/bash
# round 6, s6: N > 1 rehearsal of bench.py on ONE GPU (2 ranks over gloo sharing the card; timings
# meaningless): every world > 1 line must run without extras_error keys
set -o pipefail
mkdir -p gpurun_out/r06/s6
cd /root/repo
export BE_BENCH_BACKEND=gloo BE_BENCH_SHARED_GPU=1 PYTHONFAULTHANDLER=1
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --train-steps 3 > gpurun_out/r06/s6/rehearsal_w2.log 2>&1
rc=$?
grep '^{"metric"' gpurun_out/r06/s6/rehearsal_w2.log > gpurun_out/r06/s6/rehearsal_w2.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06/s6/rehearsal_w2.json"))
print("n_gpus", d["n_gpus"], "errors:", {k: v for k, v in d.items() if k.startswith("extras_error")})
for k in ("served_imgs_per_sec_node_c128", "finetune_cpsam_samples_per_sec", "finetune_cpsam_zero_samples_per_sec", "em_volume_voxels_per_sec", "em_volume3d_voxels_per_sec", "finetune_samples_per_sec"):
    print(k, d.get(k))
PY
exit $rc
