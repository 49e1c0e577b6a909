#!/bin/bash
# Round-4 (y): the OTU tally's bitonic exchanges by DPP -- service tests and tally phases.
set -euo pipefail
TAG=${1:-r4y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo "[gpu_r4y] done" >&2
