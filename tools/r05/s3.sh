#!/bin/bash
# round 5 step 3: CPSAM training step on the in-house GEMMs (mt) vs the library (lib), batch 8 and 1,
# alternating processes; CPSAM numerics test on mt; Cellpose-SAM inference bench on mt vs lib
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s3
mkdir -p $O
BE_CPSAM_GEMM=mt timeout -k 10 300 python -u -m pytest tests/test_cpsam_numerics_gpu.py -x -q --timeout 200 --timeout-method thread > $O/numerics_mt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/numerics_mt.log; tail -3 $O/numerics_mt.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for g in mt lib; do
    BE_CPSAM_GEMM=$g timeout -k 10 240 python -u tools/cpsam_train_bench.py --batch 8 1 --steps 15 >> $O/train_ab.jsonl 2>&1 || exit 1
  done
done
grep '"bench"' $O/train_ab.jsonl | cut -c1-200
python - > $O/infer_ab.jsonl 2>&1 <<'PY' || exit 1
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
import bench
from bioengine_worker_amd.models.cpsam import CPSAMEngine
dev = torch.device("cuda", 0)
for g in ("mt", "lib", "mt"):
    CPSAMEngine.GEMM = g
    print(json.dumps({"gemm": g, **bench.bench_cpsam_infer(dev)}), flush=True)
PY
cat $O/infer_ab.jsonl | cut -c1-300
