#!/bin/bash
# round 6, s24: where is the intermittent c = 64 tail inside the full bench? bench.py with the serving
# timeline (slow-request start times, GC pauses of the bench process)
set -o pipefail
mkdir -p gpurun_out/r06/s24
cd /root/repo
rm -f gpurun_out/r06/s24/timeline.jsonl
BE_SERVE_TIMELINE=gpurun_out/r06/s24/timeline.jsonl timeout -k 10 900 python -u bench.py --no-em > gpurun_out/r06/s24/bench.log 2>&1 || { tail -20 gpurun_out/r06/s24/bench.log; exit 1; }
grep -o '"served_[a-z0-9_]*": [0-9.]*' gpurun_out/r06/s24/bench.log | head -12
python - <<'PY'
import json
for l in open("gpurun_out/r06/s24/timeline.jsonl"):
    d = json.loads(l)
    print("c", d["concurrency"], "phase", d["phase_s"], "p99", d["p99_ms"])
    print("  slow (start s, ms):", d["slow_start_s_and_ms"][:60])
    print("  gc:", d["gc_pauses_over_2ms_s_ms_gen_collected"][:20])
PY
