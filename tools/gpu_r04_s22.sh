#!/bin/bash
# round 4 step 22: rehearsal of the driver's N-rank bench on a one-GPU box -- 3 ranks (a middle rank
# with both z-neighbours for the EM halo exchange) sharing the GPU over gloo.  Checks that every
# multi-rank line runs and rank 0 prints one JSON line; the timings mean nothing here.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=$PWD/gpurun_out/r04/s22
mkdir -p $O
BE_BENCH_BACKEND=gloo BE_BENCH_SHARED_GPU=1 timeout -k 10 1000 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 3 --steps 3 --warmup 1 --train-steps 3 --em-z 32 \
  > $O/bench_3rank.json 2> $O/bench_3rank.err || { tail -40 $O/bench_3rank.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/bench_3rank.json").read().strip().splitlines()[-1])
print({k: d[k] for k in ("metric", "value", "n_gpus", "steps")})
print("errors:", {k: v for k, v in d.items() if "error" in k})
print("keys:", sorted(d))
PY
