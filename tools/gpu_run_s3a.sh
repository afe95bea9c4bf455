set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r3s3.log 2>&1 || exit 1
for v in 0 1; do
  BE_CPSAM_SIDE_WGRAD=$v timeout -k 10 240 python -u tools/cpsam_train_bench.py --batch 1 8 --steps 20 > gpurun_out/cpsam_side_$v.jsonl 2>&1 || exit 2
done
timeout -k 10 450 python -u bench.py > gpurun_out/bench_r3s3.log 2>&1 || exit 3
