set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s31
mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "best_calls_in_the_collect or random_batch" > "$OUT/pytest.log" 2>&1 && echo done
