#!/bin/bash
# Round-4 (v): the C2 step by scorer (hybrid lane scorer / wave scorer), alternating.
set -euo pipefail
TAG=${1:-r4v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 40 --warmup 5"
for rep in 1 2 3; do
  for sv in 0 1; do
    timeout -k 10 300 $B --score-variant $sv > "$OUT/sv$sv.$rep.json" 2> "$OUT/sv$sv.$rep.err"
  done
done
echo "[gpu_r4v] done" >&2
