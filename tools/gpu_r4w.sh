#!/bin/bash
# Round-4 (w): the C2 step by the lane scorer's records per batch (4 / 8 / 16), alternating.
set -euo pipefail
TAG=${1:-r4w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 40 --warmup 5"
for rep in 1 2 3; do
  for sb in 8 16 4; do
    KGX_SCORE_BATCH=$sb timeout -k 10 300 $B > "$OUT/sb$sb.$rep.json" 2> "$OUT/sb$sb.$rep.err"
  done
done
KGX_SCORE_BATCH=16 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_score.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_score16.log" 2>&1
echo "[gpu_r4w] done" >&2
