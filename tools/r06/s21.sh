#!/bin/bash
# round 6, s21: EDT fallback with line-interleaved stacks (test + the 3-D line's stages), watershed max_local 64
set -o pipefail
mkdir -p gpurun_out/r06/s21
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_em_watershed.py tests/test_em_gpu.py -m gpu > gpurun_out/r06/s21/tests.log 2>&1 || { tail -30 gpurun_out/r06/s21/tests.log; exit 1; }
tail -2 gpurun_out/r06/s21/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/em3d_bench.py --em3d-z 64 --sweep 64:256:4 > gpurun_out/r06/s21/em3d_$r.log 2>&1 || { tail -20 gpurun_out/r06/s21/em3d_$r.log; exit 1; }
  python - "$r" <<'PY'
import json, sys
for l in open(f"gpurun_out/r06/s21/em3d_{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l); c = d["em_volume3d_config"]; t = c["stage_timings_s_rank0"]
        print("3d", round(d["em_volume3d_voxels_per_sec"] / 1e6, 1), "Mvox/s label", t["label"], t.get("split_stages"))
PY
done
