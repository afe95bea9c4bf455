#!/bin/bash
# new attention backward (variant bwd2: double-buffered tiles, folded row constants) numerics + timing
set -o pipefail
O=$PWD/gpurun_out/s4
mkdir -p $O
VD=$PWD/bioengine_worker_amd/_native/variants
BE_HIP_LIB=$VD/bwd2/libbe_hip.so timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cpsam_train_gpu.py tests/test_cpsam_numerics_gpu.py > $O/tests_bwd2.log 2>&1 || { tail -40 $O/tests_bwd2.log; exit 1; }
grep -E "passed|failed|ViT-L|loss fp32" $O/tests_bwd2.log
for r in 1 2; do
  for v in new_vform bwd2; do
    BE_HIP_LIB=$VD/$v/libbe_hip.so timeout -k 10 60 python3 tools/attn_bench.py > $O/attn_${v}_$r.jsonl 2>&1 || exit 1
    BE_HIP_LIB=$VD/$v/libbe_hip.so timeout -k 10 60 python3 tools/attn_bench.py --B 1 > $O/attn1_${v}_$r.jsonl 2>&1 || exit 1
  done
done
for f in $O/attn*.jsonl; do echo "$(basename $f) $(grep fwd $f)"; done
for r in 1 2; do
  for v in new_vform bwd2; do
    BE_HIP_LIB=$VD/$v/libbe_hip.so timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/train_${v}_$r.jsonl 2>&1 || { cat $O/train_${v}_$r.jsonl; exit 1; }
  done
done
for f in $O/train_*.jsonl; do echo $f; grep bench $f | cut -c1-130; done

# deep-level conv counters (3x3, 64-ch tiles, cin chunks of 32): where the 27-34 % MFMA time goes
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --kernel-include-regex "conv2d_nhwc_kernel" --output-format csv -d $O/convpmc -o p -- python3 $OLDPWD/tools/conv_roofline.py --mode pmc --order $O/conv_order.json > $O/convpmc.log 2>&1 || { tail $O/convpmc.log; exit 1; }
echo pmc done
echo done
