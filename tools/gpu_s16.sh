set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s16}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s16] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 120 tests/native/wave_sort_check 3000 7 > "$OUT/wave_sort.txt" 2>&1
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
for m in block sleep:20 spin sleep:50 block; do
  KGX_HOST_WAIT=$m step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,16,24 --threads 16 --seconds 3 \
     > "$OUT/lk_${m/:/_}.json" 2> "$OUT/lk_${m/:/_}.err"
done
KGX_HOST_WAIT=block step timeout -k 10 600 python3 -u -m pytest tests/test_server.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_server_block.log" 2>&1
echo "[gpu_s16] done" >&2
