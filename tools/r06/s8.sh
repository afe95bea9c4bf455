#!/bin/bash
# round 6, s8: 3-D conv path A/B on the 3-D EM line (64 x 2048^2 slab): one-launch igemm vs the
# depth-tap decomposition onto the 2-D LDS-staged kernel, for narrow layers / all layers
set -o pipefail
mkdir -p gpurun_out/r06/s8
cd /root/repo
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv3d.py -m gpu -k ztaps > gpurun_out/r06/s8/test_ztaps.log 2>&1 || { tail -30 gpurun_out/r06/s8/test_ztaps.log; exit 1; }
tail -1 gpurun_out/r06/s8/test_ztaps.log
for arm in "igemm 0" "ztaps 0" "igemm 32" "taps 0"; do
  set -- $arm
  BE_CONV3D=$1 BE_CONV3D_TAPS_MAXCIN=$2 timeout -k 10 300 python -u tools/em3d_bench.py --em3d-z 64 > gpurun_out/r06/s8/em3d_$1_$2.json 2>&1 || { tail -5 gpurun_out/r06/s8/em3d_$1_$2.json; exit 1; }
  echo "$arm $(grep em_volume3d gpurun_out/r06/s8/em3d_$1_$2.json | python -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['em_volume3d_config']; print(round(d['em_volume3d_voxels_per_sec']/1e6,1), c['stage_timings_s_rank0']['inference'])")"
done
