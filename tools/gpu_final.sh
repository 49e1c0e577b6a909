#!/bin/bash
# A round's closing pass: the closing check, then the two-rank rehearsal of
# bench.py's multi-rank path (canary on every rank).  bash tools/gpu_final.sh TAG
set -euo pipefail
TAG=${1:-final}
bash tools/gpu_check.sh "$TAG"
bash tools/rehearse_ranks.sh "${TAG}_ranks"
echo "[gpu_final] done" >&2
