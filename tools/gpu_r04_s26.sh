#!/bin/bash
# round 4 step 26: IVF full-probe failure -- uniqueness of torch.topk probe lists on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s26
mkdir -p $O
timeout -k 10 200 python3 tools/topk_probe_check.py > $O/topk.log 2>&1 || { tail -20 $O/topk.log; exit 1; }
cat $O/topk.log
