#!/bin/bash
# Round-4 (m): host path vs the number of hardware queues per process (streams share them FIFO).
set -euo pipefail
TAG=${1:-r4m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for q in 4 8 16; do
  for u in 1 0; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6,8 --copy 1 --hits16 1 --stream 1 \
        --rec12 1 --score 0 --want 11 --opt host_upload_stream=$u > "$OUT/hp_q${q}_up$u.json" 2> "$OUT/hp_q${q}_up$u.err"
  done
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 0 --want 11 --timing > "$OUT/hp_q16_timing.json" 2> "$OUT/hp_q16_timing.err"
echo "[gpu_r4m] done" >&2
