#!/bin/bash
# The -m gpu suite and smoke on the current tree.  bash tools/gpu_tests.sh TAG
set -euo pipefail
TAG=${1:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "[gpu_tests] done" >&2
