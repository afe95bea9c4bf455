#!/bin/bash
# CPSAM fine-tune A/B on one box: tuned hipBLASLt epilogue GEMMs (ops/gemm.py) vs PyTorch GEMMs,
# interleaved so box drift does not bias either side; per-GEMM table for both.
set -o pipefail
O=$PWD/gpurun_out/cpsam_ab
mkdir -p $O
timeout -k 10 180 python3 tools/vit_gemm_bench.py --B 8 > $O/gemm_b8.jsonl 2>&1 || { cat $O/gemm_b8.jsonl; exit 1; }
timeout -k 10 120 python3 tools/vit_gemm_bench.py --B 1 > $O/gemm_b1.jsonl 2>&1 || { cat $O/gemm_b1.jsonl; exit 1; }
grep total $O/gemm_b8.jsonl $O/gemm_b1.jsonl
for r in 1 2; do
  timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/lt_$r.jsonl 2>&1 || { cat $O/lt_$r.jsonl; exit 1; }
  BE_LT=0 timeout -k 10 240 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 30 > $O/torch_$r.jsonl 2>&1 || { cat $O/torch_$r.jsonl; exit 1; }
  cat $O/lt_$r.jsonl $O/torch_$r.jsonl | grep bench
done
echo done
