#!/bin/bash
# round 4 step 16: AdamW kernel A/B (ViT-L-sized flat buffer)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/s16
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_adamw_variants.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/adamw_ab.py > $O/adamw_ab.jsonl 2>&1 || { tail -20 $O/adamw_ab.jsonl; exit 1; }
grep '^{' $O/adamw_ab.jsonl
