#!/bin/bash
# Round-4 (al): the host path's streamed chunks under rocprofv3 --kernel-trace (what fills a chunk's
# scan + gather segment beside the other context's probe).
set -euo pipefail
TAG=${1:-r4al}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/kt" -o kt \
    -- python3 "$R/tools/host_path_probe.py" --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
      --rec12 1 --taper 1 --stage 8 --score 0 --want 11 > "$OUT/kt.json" 2> "$OUT/kt.err")
echo "[gpu_r4al] done" >&2
