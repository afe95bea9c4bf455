#!/bin/bash
# round 6, s21: EDT fallback with line-interleaved stacks and the 32 x 32-tile watershed: GPU tests,
# then the 3-D line's stages (64 x 2048^2 slab) with BE_WS_TILE 32 / 16
set -o pipefail
mkdir -p gpurun_out/r06/s21
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_em_watershed.py tests/test_em_gpu.py -m gpu > gpurun_out/r06/s21/tests.log 2>&1 || { tail -30 gpurun_out/r06/s21/tests.log; exit 1; }
tail -2 gpurun_out/r06/s21/tests.log
for arm in 32 16 32 16; do
  BE_WS_TILE=$arm timeout -k 10 300 python -u tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > gpurun_out/r06/s21/em3d_ws$arm.log 2>&1 || { tail -20 gpurun_out/r06/s21/em3d_ws$arm.log; exit 1; }
  python - "$arm" <<'PY'
import json, sys
for l in open(f"gpurun_out/r06/s21/em3d_ws{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]; t = c["stage_timings_s_rank0"]
        print("ws", sys.argv[1], round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s label", t["label"], t.get("split_stages"))
PY
done
