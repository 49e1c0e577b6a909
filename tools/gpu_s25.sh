set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s25}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s25] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest $(grep -ln "rollup\|lookup" tests/test_gpu*.py tests/test_server.py) -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step timeout -k 10 900 python3 bench.py --no-cpu-baseline --no-host-path --no-pool > "$OUT/bench.json" 2> "$OUT/bench.err"
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,16 --wait sleep:20 --one-wait > "$OUT/pp_one.json" 2> "$OUT/pp_one.err"
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 --seconds 3 > "$OUT/lk.json" 2> "$OUT/lk.err"
echo "[gpu_s25] done" >&2
