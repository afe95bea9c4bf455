#!/bin/bash
# round 4 step 7: CPSAM step A/B of the GEMM backends (library vs per-shape auto choice)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
for g in lib auto; do
  BE_CPSAM_GEMM=$g timeout -k 10 300 python -u tools/cpsam_train_bench.py --batch 1 8 --steps 20 > gpurun_out/r04/s7_cpsam_$g.jsonl 2>&1 || { tail -20 gpurun_out/r04/s7_cpsam_$g.jsonl; exit 1; }
  grep '^{' gpurun_out/r04/s7_cpsam_$g.jsonl | cut -c1-400
done
