#!/bin/bash
# Round-4 (q): the C2 step vs its probe -- probes on one image stream at high
# priority (KGX_PROBE_PRIORITY=1) or normal, and the default per-context chain.
set -euo pipefail
TAG=${1:-r4q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 40 --warmup 5"
for rep in 1 2 3; do
  timeout -k 10 300 $B > "$OUT/default.$rep.json" 2> "$OUT/default.$rep.err"
  timeout -k 10 300 $B --probe-stream 1 > "$OUT/pstream.$rep.json" 2> "$OUT/pstream.$rep.err"
  KGX_PROBE_PRIORITY=1 timeout -k 10 300 $B --probe-stream 1 > "$OUT/pstream_hi.$rep.json" 2> "$OUT/pstream_hi.$rep.err"
done
echo "[gpu_r4q] done" >&2
