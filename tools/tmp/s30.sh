set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s30
mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && echo done
