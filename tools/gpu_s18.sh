set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s18}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s18] stop: rc $rc from $*" >&2; exit $rc; fi; }
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
export KGX_HOST_WAIT=sleep:20
run() { tag=$1; shift; step env "$@" timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24 --threads 16 --seconds 3 > "$OUT/lk_$tag.json" 2> "$OUT/lk_$tag.err"; }
run base X=1
run batch KGX_LOOKUP_BATCH=1
run unchained KGX_SERVER_PROBE_SERIALIZE=0
run onewait KGX_LOOKUP_ONE_WAIT=1
KGX_HOST_WAIT=sleep:20 step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24,32 --threads 24 --seconds 3 > "$OUT/lk_t24.json" 2> "$OUT/lk_t24.err"
echo "[gpu_s18] done" >&2
