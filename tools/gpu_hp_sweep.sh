#!/bin/bash
# The host path's schedule on the current tree: chunks x taper x staging threads, and the bench's own leg.
set -euo pipefail
TAG=${1:-hp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,5,6,8 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --taper 0,1 --stage 4,8 --score 0 --want 11 > "$OUT/sweep.json" 2> "$OUT/sweep.err"
echo "[gpu_hp_sweep] done" >&2
