#!/bin/bash
# round 5 step 46: __graft_entry__.smoke() on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -3
