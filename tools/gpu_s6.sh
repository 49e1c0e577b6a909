set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s6}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_plan.py -m gpu -x -v --timeout 250 --timeout-method thread > "$OUT/pytest_plan.log" 2>&1 || true
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_svc.py -m gpu -x -q --timeout 250 --timeout-method thread -k "otu or wave_sort" -s > "$OUT/pytest_otu.log" 2>&1 || true
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
