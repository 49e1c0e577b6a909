#!/bin/bash
# Round-4: the service reading its slot's residues 16 bytes per thread -- tests and phases.
set -euo pipefail
TAG=${1:-r4aa}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade.json" 2> "$OUT/facade.err"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16 KGX_SVC_DEBUG=1 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_dbg.json" 2> "$OUT/facade_dbg.err"
echo "[gpu] done" >&2
