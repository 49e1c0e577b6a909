#!/bin/bash
# What the driver runs at a round's end, on the current tree: the -m gpu suite, smoke, the default bench line.
set -euo pipefail
TAG=${1:-last}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 900 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "[gpu_last] done" >&2
