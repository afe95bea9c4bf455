#!/bin/bash
# round 5 step 26: mask stage round 2 (bit-row hole filling for boxes up to 256 x 128, follow-flows
# tile size by batch) and the EM labelling passes (bounded-search EDT-3D, active-tile watershed):
# tests, EM stage timings A/B, headline + b1 A/B, EM volume bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r05/s26
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cellpose_gpu.py tests/test_em_watershed.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "== tests $(tail -1 $O/tests.log)"
for ws in 1 0; do
  BE_WS_ACTIVE=$ws timeout -k 10 200 python3 -u tools/em_split_profile.py 256 > $O/em_split_ws$ws.json 2> $O/em_split_ws$ws.err || { tail -20 $O/em_split_ws$ws.err; exit 1; }
  echo "ws_active=$ws $(cat $O/em_split_ws$ws.json)"
done
for r in 1 2; do
  for cfg in base follow_xcd fill_lds; do
    case $cfg in
      base) E="";;
      follow_xcd) E="BIOENGINE_FOLLOW_ENTRY=be_cp_follow_flows_xcd";;
      fill_lds) E="BE_FILL_WAVE=0";;
    esac
    env $E timeout -k 10 200 python -u tools/headline_ab.py > $O/head_${cfg}_$r.json 2>>$O/head_ab.err || exit 1
    echo "$cfg $(cut -c1-100 $O/head_${cfg}_$r.json)"
  done
done
timeout -k 10 400 python3 -u tools/em_volume_bench.py --z 256 --split-touching > $O/em_volume.json 2> $O/em_volume.err || { tail -20 $O/em_volume.err; exit 1; }
cut -c1-900 $O/em_volume.json
