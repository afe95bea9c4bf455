#!/bin/bash
# attention backward A/B on one box: current (dkv DMA + sched fence), s14 codegen, dq DMA variant
set -o pipefail
R=$PWD
O=$R/gpurun_out/s16
mkdir -p $O
VD=$R/bioengine_worker_amd/_native/variants/dqdma/libbe_hip.so
VS=$R/bioengine_worker_amd/_native/variants/s14/libbe_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py -k attn_bwd > $O/test_base.log 2>&1 || { tail -30 $O/test_base.log; exit 1; }
tail -1 $O/test_base.log
BE_HIP_LIB=$VD timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py -k attn_bwd > $O/test_dq.log 2>&1 || { tail -30 $O/test_dq.log; exit 1; }
tail -1 $O/test_dq.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py --iters 30 | sed 's/^/cur /' >> $O/attn.jsonl || exit 1
  BE_HIP_LIB=$VS timeout -k 10 120 python tools/attn_bench.py --iters 30 | sed 's/^/s14 /' >> $O/attn.jsonl || exit 1
  BE_HIP_LIB=$VD timeout -k 10 120 python tools/attn_bench.py --iters 30 | sed 's/^/dqdma /' >> $O/attn.jsonl || exit 1
done
timeout -k 10 120 python tools/attn_bench.py --iters 30 --B 1 | sed "s/^/cur /" >> $O/attn.jsonl || exit 1
BE_HIP_LIB=$VD timeout -k 10 120 python tools/attn_bench.py --iters 30 --B 1 | sed "s/^/dqdma /" >> $O/attn.jsonl || exit 1
cat $O/attn.jsonl
echo done
