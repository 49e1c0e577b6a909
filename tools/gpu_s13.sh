set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s13}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_s13] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 600 python3 -u -m pytest tests/test_server.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > "$OUT/pytest_server.log" 2>&1
P="/lookup?family_mode=1&find_best_match=1"
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,8,16 --threads 16 > "$OUT/lk_t16_batch.json" 2> "$OUT/lk_t16_batch.err"
export KGX_LOOKUP_BATCH=0
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16_nobatch.json" 2> "$OUT/lk_t16_nobatch.err"
unset KGX_LOOKUP_BATCH
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24 --threads 24 > "$OUT/lk_t24_batch.json" 2> "$OUT/lk_t24_batch.err"
echo "[gpu_s13] done" >&2
