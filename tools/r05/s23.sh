#!/bin/bash
# round 5 steps 2+3 in one box session (the pool is scarce): gemm_mt numerics, the per-shape sweep,
# fp8 / CPSAM-engine / conv3d GPU tests, ViT qkv A/B, CPSAM training A/B (mt vs lib), Cellpose-SAM
# inference bench.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s23
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_mt.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; tail -12 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u tools/gemm_mt_bench.py --table --rounds 5 > $O/sweep.jsonl 2>&1
rc=$?; echo "sweep rc=$rc" >> $O/sweep.jsonl; grep -A40 "^TABLE" $O/sweep.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_fp8.py tests/test_transformer_gpu.py tests/test_conv3d.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests2.log; tail -5 $O/tests2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/vit_qkv_ab.py > $O/vit_qkv_ab.jsonl 2>&1 || exit 1
cat $O/vit_qkv_ab.jsonl | tail -3
BE_CPSAM_GEMM=mt timeout -k 10 300 python -u -m pytest tests/test_cpsam_numerics_gpu.py -x -q --timeout 200 --timeout-method thread > $O/numerics_mt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/numerics_mt.log; tail -3 $O/numerics_mt.log
[ $rc -eq 0 ] || exit $rc
for g in mt lib mt lib; do
  BE_CPSAM_GEMM=$g timeout -k 10 240 python -u tools/cpsam_train_bench.py --batch 8 1 --steps 15 >> $O/train_ab.jsonl 2>&1 || exit 1
done
grep '"bench"' $O/train_ab.jsonl | cut -c1-160
timeout -k 10 400 python - > $O/infer_ab.jsonl 2>&1 <<'PY' || exit 1
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
import bench
from bioengine_worker_amd.models.cpsam import CPSAMEngine
dev = torch.device("cuda", 0)
for g in ("mt", "lib", "mt"):
    CPSAMEngine.GEMM = g
    print(json.dumps({"gemm": g, **bench.bench_cpsam_infer(dev)}), flush=True)
PY
cut -c1-300 $O/infer_ab.jsonl
