#!/bin/bash
# Round-4 (l): host path with chunk uploads on their own stream (host_upload_stream 1 / 0).
set -euo pipefail
TAG=${1:-r4l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "host or stream or compact or chunk or pool" > "$OUT/pytest.log" 2>&1
for rep in 1 2; do
  for u in 1 0; do
    timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6,8 --copy 1 --hits16 1 --stream 1 \
        --rec12 1 --score 0 --want 11 --opt host_upload_stream=$u > "$OUT/host_path_up$u.$rep.json" 2> "$OUT/host_path_up$u.$rep.err"
  done
done
timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 0 --want 11 --timing > "$OUT/host_path_timing.json" 2> "$OUT/host_path_timing.err"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "[gpu_r4l] done" >&2
