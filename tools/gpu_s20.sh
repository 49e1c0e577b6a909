set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s20}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s20] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest $(grep -ln "rollup\|lookup" tests/test_gpu*.py tests/test_server.py) -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,16,24 --wait sleep:20 > "$OUT/pp_two.json" 2> "$OUT/pp_two.err"
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,16,24 --wait sleep:20 --one-wait > "$OUT/pp_one.json" 2> "$OUT/pp_one.err"
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp KGX_HOST_WAIT=sleep:20
step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24 --threads 16 --seconds 3 > "$OUT/lk_two.json" 2> "$OUT/lk_two.err"
KGX_LOOKUP_ONE_WAIT=1 step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24 --threads 16 --seconds 3 > "$OUT/lk_one.json" 2> "$OUT/lk_one.err"
echo "[gpu_s20] done" >&2
