#!/bin/bash
# Round-4 (am): the host path by copy workgroups (device stores into mapped memory slow every
# kernel beside them, r4al) and DMA copies, alternating.
set -euo pipefail
TAG=${1:-r4am}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for rep in 1 2; do
  timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --copy-blocks 4,8,16,32,64 \
      --hits16 1 --stream 1 --rec12 1 --taper 1 --stage 8 --score 0 --want 11 > "$OUT/blocks.$rep.json" 2> "$OUT/blocks.$rep.err"
  timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 0 \
      --hits16 1 --stream 1 --rec12 1 --taper 1 --stage 8 --score 0 --want 11 > "$OUT/dma.$rep.json" 2> "$OUT/dma.$rep.err"
done
echo "[gpu_r4am] done" >&2
