#!/bin/bash
# CPSAM A/B (tests + attention/step benches, tools/gpu_attn_ab.sh) then a kernel-trace profile at batch ${B:-1}.
set -o pipefail
bash tools/gpu_attn_ab.sh || exit $?
B=${B:-1} bash tools/gpu_prof_cpsam.sh
