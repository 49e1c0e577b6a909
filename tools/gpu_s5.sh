set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s5}
mkdir -p "$OUT"
cd "$R"
P="/lookup?family_mode=1&find_best_match=1"
KGX_LOOKUP_ONE_WAIT=1 timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 8,16 --threads 8 > "$OUT/lk_t8_w1.json" 2> "$OUT/lk_t8_w1.err"
KGX_LOOKUP_ONE_WAIT=0 timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 8,16 --threads 8 > "$OUT/lk_t8_w0.json" 2> "$OUT/lk_t8_w0.err"
KGX_LOOKUP_ONE_WAIT=1 timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16_w1.json" 2> "$OUT/lk_t16_w1.err"
