#!/bin/bash
# Round-4 (t): streamed chunks on the wave scorer -- parity, then the bench's host path.
set -euo pipefail
TAG=${1:-r4t}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_full_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
B="python3 bench.py --no-cpu-baseline --no-microbench --no-canary --steps 10 --warmup 3"
for rep in 1 2 3; do
  timeout -k 10 300 $B > "$OUT/bench.$rep.json" 2> "$OUT/bench.$rep.err"
done
echo "[gpu_r4t] done" >&2
