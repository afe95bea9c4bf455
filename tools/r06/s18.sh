#!/bin/bash
# round 6, s18: the sub-pixel concat source (INMODE 6) and the unpadded 16-channel 3-D layers: GPU tests,
# then the 2-D EM line A/B (BE_UNET_LAZY) and the 3-D line A/B (BE_CONV3D_NARROW), 64 x 2048^2 slabs
set -o pipefail
mkdir -p gpurun_out/r06/s18
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_deferred_fusion.py tests/test_conv3d.py -m gpu > gpurun_out/r06/s18/tests.log 2>&1 || { tail -30 gpurun_out/r06/s18/tests.log; exit 1; }
tail -2 gpurun_out/r06/s18/tests.log
for arm in 1 0 1 0; do
  BE_UNET_LAZY=$arm timeout -k 10 300 python -u tools/em2d_bench.py --em-z 64 --sweep 768:64:16 > gpurun_out/r06/s18/em2d_lazy$arm.log 2>&1 || { tail -20 gpurun_out/r06/s18/em2d_lazy$arm.log; exit 1; }
  python - "$arm" <<'PY'
import json, sys
for l in open(f"gpurun_out/r06/s18/em2d_lazy{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume_config"]; t = c["stage_timings_s_rank0"]
        print("lazy", sys.argv[1], round(d["em_volume_voxels_per_sec"] / 1e6, 1), "Mvox/s inference", t["inference"], "label", t["label"])
PY
done
for arm in n1c0 n1c1 n0c0 n1c0 n1c1; do
  nar=${arm:1:1}; c16=${arm:3:1}
  BE_CONV3D_NARROW=$nar BE_CONV3D_CK16=$c16 timeout -k 10 300 python -u tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > gpurun_out/r06/s18/em3d_$arm.log 2>&1 || { tail -20 gpurun_out/r06/s18/em3d_$arm.log; exit 1; }
  python - "$arm" <<'PY'
import json, sys
for l in open(f"gpurun_out/r06/s18/em3d_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]; t = c["stage_timings_s_rank0"]
        print("3d", sys.argv[1], round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s inference", t["inference"], "label", t["label"])
PY
done
