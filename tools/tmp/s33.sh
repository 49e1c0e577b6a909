set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s33
mkdir -p "$OUT"; cd "$R"
timeout -k 10 120 tests/native/wave_sort_check 3000 7 > "$OUT/wave_sort.txt" 2>&1
echo done
