set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s24}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s24] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest tests/test_server.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
KGX_TEXT_CLOCKS=1 step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,16 --threads 16 --seconds 3 > "$OUT/lk_clocks.json" 2> "$OUT/lk_clocks.err"
step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,16,24 --threads 16 --seconds 3 > "$OUT/lk.json" 2> "$OUT/lk.err"
echo "[gpu_s24] done" >&2
