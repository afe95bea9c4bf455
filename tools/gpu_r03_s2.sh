#!/bin/bash
# Round-3 session-2 check: attention variants (HEAD kernel / VGPR-form build / new forward loop /
# new + VGPR-form) numerics + timing, GEMM A/B with the GELU-backward on the HIP kernel, CPSAM step.
set -o pipefail
O=$PWD/gpurun_out/s2
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
BE_HIP_LIB=$VD/new_vform/libbe_hip.so timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cpsam_train_gpu.py tests/test_gemm_lt_gpu.py > $O/tests_new_vform.log 2>&1 || { tail -40 $O/tests_new_vform.log; exit 1; }
tail -2 $O/tests_new_vform.log
for r in 1 2; do
  for v in base vform new new_vform; do
    L=$VD/$v/libbe_hip.so; [ $v = base ] && L=$PWD/bioengine_worker_amd/_native/libbe_hip.so
    BE_HIP_LIB=$L timeout -k 10 60 python3 tools/attn_bench.py > $O/attn_${v}_$r.jsonl 2>&1 || exit 1
    BE_HIP_LIB=$L timeout -k 10 60 python3 tools/attn_bench.py --B 1 > $O/attn1_${v}_$r.jsonl 2>&1 || exit 1
  done
done
for f in $O/attn*.jsonl; do echo "$(basename $f) $(grep fwd $f)"; done
timeout -k 10 180 python3 tools/vit_gemm_bench.py --B 8 > $O/gemm_b8.jsonl 2>&1 || exit 1
timeout -k 10 120 python3 tools/vit_gemm_bench.py --B 1 > $O/gemm_b1.jsonl 2>&1 || exit 1
grep total $O/gemm_b*.jsonl
for r in 1 2; do
  timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/lt_$r.jsonl 2>&1 || { cat $O/lt_$r.jsonl; exit 1; }
  BE_HIP_LIB=$VD/new_vform/libbe_hip.so timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/ltv_$r.jsonl 2>&1 || { cat $O/ltv_$r.jsonl; exit 1; }
  BE_LT=0 timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/torch_$r.jsonl 2>&1 || { cat $O/torch_$r.jsonl; exit 1; }
done
for f in $O/lt_*.jsonl $O/ltv_*.jsonl $O/torch_*.jsonl; do echo $f; grep bench $f | cut -c1-160; done
echo done
