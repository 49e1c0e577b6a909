#!/bin/bash
# Round-4 (an): the streamed chunks' copies by DMA (host_stream_dma) vs device stores -- parity,
# then the host path alternating.
set -euo pipefail
TAG=${1:-r4an}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
for rep in 1 2; do
  for dma in 1 0; do
    timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 5,6,8 --copy 1 --hits16 1 --stream 1 \
        --rec12 1 --taper 1 --stage 8 --score 0 --want 11 --opt host_stream_dma=$dma > "$OUT/dma$dma.$rep.json" 2> "$OUT/dma$dma.$rep.err"
  done
done
timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --taper 1 --stage 8 --score 0 --want 11 --opt host_stream_dma=1 --timing > "$OUT/dma1.timing.json" 2> "$OUT/dma1.timing.err"
echo "[gpu_r4an] done" >&2
