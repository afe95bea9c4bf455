set -o pipefail
mkdir -p gpurun_out/attn2
timeout -k 10 200 python -u -m pytest tests/test_cpsam_train_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/attn2/tests.log 2>&1 || { tail -20 gpurun_out/attn2/tests.log; exit 1; }
tail -3 gpurun_out/attn2/tests.log
timeout -k 10 120 python3 tools/attn_bench.py > gpurun_out/attn2/time.jsonl 2>&1 || exit $?
timeout -k 10 120 python3 tools/attn_bench.py --B 1 >> gpurun_out/attn2/time.jsonl 2>&1 || exit $?
grep '^{' gpurun_out/attn2/time.jsonl
timeout -k 10 300 python3 tools/cpsam_train_bench.py --batch 8 --steps 10 --warmup 3 > gpurun_out/attn2/train.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/cpsam_train_bench.py --batch 1 --steps 20 --warmup 3 >> gpurun_out/attn2/train.log 2>&1 || exit $?
grep '^{' gpurun_out/attn2/train.log
