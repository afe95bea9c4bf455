#!/bin/bash
# round 5 step 30 = s28 (cellpose tests, batch-1 anatomy) + s29 (mask kernels beside the convs A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r05/s28.sh || exit 1
bash tools/r05/s29.sh || exit 1
