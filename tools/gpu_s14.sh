set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s14}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s14] stop: rc $rc from $*" >&2; exit $rc; fi; }
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 --seconds 3 \
   > "$OUT/lk.json" 2> "$OUT/lk.err"
step timeout -k 10 500 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 --seconds 3 \
   --allow-failures --server-prefix "rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/srv -o srv --" > "$OUT/lk_trace.json" 2> "$OUT/lk_trace.err"
step timeout -k 10 120 python3 tools/server_trace.py "$OUT/srv" 1 > "$OUT/srv_trace.json"
find "$OUT/srv" -name "*kernel_trace.csv" -delete
echo "[gpu_s14] done" >&2
