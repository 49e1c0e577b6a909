#!/bin/bash
# Round-4 (f): the call service's pair sort timed twice on copies (cold code, warm code).
set -euo pipefail
TAG=${1:-r4f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo "[gpu_r4f] done" >&2
