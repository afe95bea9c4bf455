#!/bin/bash
# round 6, s3: 3-D kernels + CPSAM neck on HIP (tests), then the 3-D EM line at config scale
set -o pipefail
mkdir -p gpurun_out/r06/s3
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv3d.py tests/test_cpsam_numerics_gpu.py tests/test_cpsam_train_gpu.py -m gpu > gpurun_out/r06/s3/tests.log 2>&1 || { tail -40 gpurun_out/r06/s3/tests.log; exit 1; }
tail -3 gpurun_out/r06/s3/tests.log
timeout -k 10 400 python -u tools/em3d_bench.py --em3d-z 64 --em3d-yx 2048 > gpurun_out/r06/s3/em3d_z64.json 2>&1 || { tail -20 gpurun_out/r06/s3/em3d_z64.json; exit 1; }
grep em_volume3d gpurun_out/r06/s3/em3d_z64.json
timeout -k 10 500 python -u tools/em3d_bench.py > gpurun_out/r06/s3/em3d_full.json 2>&1 || { tail -20 gpurun_out/r06/s3/em3d_full.json; exit 1; }
grep em_volume3d gpurun_out/r06/s3/em3d_full.json
