#!/bin/bash
# add + LayerNorm with every load ahead of the stores (main) vs the committed kernel (variants/base)
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s33
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpsam_train_gpu.py tests/test_fp8.py -m gpu > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in base main base main; do
  if [ $v = base ]; then L=$R/bioengine_worker_amd/_native/variants/base/libbe_hip.so; else L=$R/bioengine_worker_amd/_native/libbe_hip.so; fi
  BE_HIP_LIB=$L timeout -k 10 200 python tools/cpsam_train_bench.py --batch 8 --steps 20 > $O/train_$v.jsonl 2>&1 || { tail $O/train_$v.jsonl; exit 1; }
  BE_HIP_LIB=$L timeout -k 10 200 python -c "import bench, torch; print('vit_fp8', round(bench.bench_vit_embed(torch.device('cuda')), 1))" > $O/vit_$v.txt 2>&1 || { tail $O/vit_$v.txt; exit 1; }
  echo $v $(grep bench $O/train_$v.jsonl | python3 -c "import json,sys; print([json.loads(l)['ms_per_step'] for l in sys.stdin])") $(grep vit_fp8 $O/vit_$v.txt)
done
echo done
