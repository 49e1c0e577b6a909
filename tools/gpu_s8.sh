# HTTP family /lookup A/B, the per-sequence facade, the two-rank rehearsal.
# A test or bench failure (rc 1) lets later steps run; a fault, abort or
# time limit ends the script.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s8}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_s8] stop: rc $rc from $*" >&2; exit $rc; fi; }
P="/lookup?family_mode=1&find_best_match=1"
export KGX_LOOKUP_ONE_WAIT=1
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 8,16 --threads 8 > "$OUT/lk_t8_w1.json" 2> "$OUT/lk_t8_w1.err"
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16_w1.json" 2> "$OUT/lk_t16_w1.err"
export KGX_LOOKUP_ONE_WAIT=0
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16_w0.json" 2> "$OUT/lk_t16_w0.err"
unset KGX_LOOKUP_ONE_WAIT
export KGX_LINE_INDEX=36 KGX_FACADE_BESIDE=8
step timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
unset KGX_LINE_INDEX KGX_FACADE_BESIDE
step timeout -k 10 700 bash tools/rehearse_ranks.sh "$(basename "$OUT")/ranks"
echo "[gpu_s8] done" >&2
