#!/bin/bash
# Round-3 CPSAM measurements: fused/tuned GEMM tests, numerics tests (ViT-L block shapes, 50-step
# loss curve), attention and GEMM micro-benchmarks, the fine-tune step with and without the
# hipBLASLt epilogue path, kernel stats of the B=8 step.
set -o pipefail
R=$PWD
O=$R/gpurun_out/cpsam_r03
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gemm_lt_gpu.py > $O/gemm_tests.log 2>&1 || { tail -40 $O/gemm_tests.log; exit 1; }
tail -3 $O/gemm_tests.log
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_cpsam_numerics_gpu.py > $O/numerics.log 2>&1 || { tail -40 $O/numerics.log; exit 1; }
grep -E "ViT-L blocks|loss fp32|passed|failed" $O/numerics.log
timeout -k 10 120 python3 tools/vit_gemm_bench.py --B 8 > $O/gemm_b8.jsonl 2>&1 || exit $?
cat $O/gemm_b8.jsonl
timeout -k 10 300 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 20 > $O/train_lt.jsonl 2>&1 || exit $?
BE_LT=0 timeout -k 10 300 python3 tools/cpsam_train_bench.py --batch 8 1 --steps 20 > $O/train_torch.jsonl 2>&1 || exit $?
cat $O/train_lt.jsonl $O/train_torch.jsonl
timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_b8.jsonl 2>&1 || exit $?
cat $O/attn_b8.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o cpsam -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit $?
tail -3 $O/prof.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $O/attn_pmc -o sq -- python3 $R/tools/attn_bench.py --iters 2 > $O/attn_pmc.log 2>&1 || exit $?
echo done
