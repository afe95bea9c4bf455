#!/bin/bash
# round 6, s11: where is the c = 64 tail? request timeline + GC pauses of the bench process
set -o pipefail
mkdir -p gpurun_out/r06/s11
cd /root/repo
rm -f gpurun_out/r06/s11/timeline.jsonl
timeout -k 10 300 python -u tools/serve_bench.py --concurrency 1,64 --seconds 4 --timeline gpurun_out/r06/s11/timeline.jsonl > gpurun_out/r06/s11/serve.log 2>&1 || { tail -20 gpurun_out/r06/s11/serve.log; exit 1; }
grep '^{' gpurun_out/r06/s11/serve.log | tail -4
python - <<'PY'
import json
for l in open("gpurun_out/r06/s11/timeline.jsonl"):
    d = json.loads(l)
    print("c", d["concurrency"], "phase", d["phase_s"], "p99", d["p99_ms"])
    print("  slow (start s, ms):", d["slow_start_s_and_ms"][:40])
    print("  gc:", d["gc_pauses_over_2ms_s_ms_gen_collected"][:20])
PY
