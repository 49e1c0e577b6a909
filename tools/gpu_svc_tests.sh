#!/bin/bash
# The call-service and facade GPU tests alone.  bash tools/gpu_svc_tests.sh TAG
set -euo pipefail
TAG=${1:-svc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
echo "[gpu_svc_tests] done" >&2
