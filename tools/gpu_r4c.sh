#!/bin/bash
# Round-4 measurements (c): the lock-free service entry and register OTU
# tally; the native beside test; the host path's chunk pipeline on the host's
# and the device's clocks.  bash tools/gpu_r4c.sh TAG
set -euo pipefail
TAG=${1:-r4c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py -m gpu -x -q -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade.json" 2> "$OUT/facade.err"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16 KGX_SVC_DEBUG=1 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_dbg.json" 2> "$OUT/facade_dbg.err"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
timeout -k 10 600 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 1 --want 11 --timing > "$OUT/host_path_timing.json" 2> "$OUT/host_path_timing.err"
echo "[gpu_r4c] done" >&2
