#!/bin/bash
# Round-4 measurements (e): the one-wave std::sort replay timed alone; the
# OTU tally (register list, sort past 8 values).  bash tools/gpu_r4e.sh TAG
set -euo pipefail
TAG=${1:-r4e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 tests/native/wave_sort_check 3000 7 > "$OUT/wave_sort.txt" 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py -m gpu -x -q -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo "[gpu_r4e] done" >&2
