#!/bin/bash
# Round-4 (ao): r4am (copy workgroups) and r4an (DMA chunk copies) in one call.
set -euo pipefail
TAG=${1:-r4ao}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_r4an.sh "$TAG"
OUT=$R/gpurun_out/$TAG
timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --copy-blocks 8,16,32,64 \
    --hits16 1 --stream 1 --rec12 1 --taper 1 --stage 8 --score 0 --want 11 > "$OUT/blocks.json" 2> "$OUT/blocks.err"
echo "[gpu_r4ao] done" >&2
