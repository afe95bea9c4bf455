set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cpnet_engine_gpu.py tests/test_cpsam_train_gpu.py tests/test_cellpose_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gn_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gn_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/gn_tests.log | head -30; exit $rc; }
timeout -k 10 600 python -u bench.py --no-served > gpurun_out/bench_gn.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gn.log; exit $rc
