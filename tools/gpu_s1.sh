set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s1
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python3 bench.py --no-host-path --no-lookup --no-pool > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_line_index.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
