#!/bin/bash
# Round-4 (s): the call service's phases incl. the closing fence and the device's whole part.
set -euo pipefail
TAG=${1:-r4s}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16 KGX_SVC_DEBUG=1 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_dbg.json" 2> "$OUT/facade_dbg.err"
echo "[gpu_r4s] done" >&2
