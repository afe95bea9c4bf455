#!/bin/bash
# round 6, s25: every batch size 1..32 prewarmed: the whole GPU suite, then bench.py --no-em with the
# serving timeline (is the intermittent c = 64 tail gone?)
set -o pipefail
mkdir -p gpurun_out/r06/s25
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/s25/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06/s25/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06/s25/gpu_tests.log
rm -f gpurun_out/r06/s25/timeline.jsonl
BE_SERVE_TIMELINE=gpurun_out/r06/s25/timeline.jsonl timeout -k 10 900 python -u bench.py --no-em > gpurun_out/r06/s25/bench.log 2>&1 || { tail -20 gpurun_out/r06/s25/bench.log; exit 1; }
grep -o '"served_[a-z0-9_]*": [0-9.]*' gpurun_out/r06/s25/bench.log | head -12
grep -o '"router[^}]*}[^}]*}' gpurun_out/r06/s25/bench.log | head -2
python - <<'PY'
import json
for l in open("gpurun_out/r06/s25/timeline.jsonl"):
    d = json.loads(l)
    print("c", d["concurrency"], "phase", d["phase_s"], "p99", d["p99_ms"])
    print("  slow (start s, ms):", d["slow_start_s_and_ms"][:30])
PY
