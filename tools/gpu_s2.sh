set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s2}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_svc.py -m gpu -x -q --timeout 200 --timeout-method thread -k stall > "$OUT/pytest_svc.log" 2>&1
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_full_scale.py tests/test_gpu_lookup_pool.py tests/test_gpu_multi.py -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_full.log" 2>&1
