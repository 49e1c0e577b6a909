set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s3}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_full_scale.py tests/test_gpu_lookup_pool.py tests/test_gpu_multi.py tests/test_gpu_line_index.py -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/pytest_full.log" 2>&1
