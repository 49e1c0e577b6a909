set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s11}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_s11] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_svc.py -m gpu -q --timeout 250 --timeout-method thread -p no:cacheprovider -s -k "otu or wave_sort" > "$OUT/pytest.log" 2>&1
export KGX_SVC_DEBUG=1
step timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
unset KGX_SVC_DEBUG
P="/lookup?family_mode=1&find_best_match=1"
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16.json" 2> "$OUT/lk_t16.err"
export KGX_SERVER_PROBE_SERIALIZE=0
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16 --threads 16 > "$OUT/lk_t16_unchained.json" 2> "$OUT/lk_t16_unchained.err"
step timeout -k 10 400 python3 tools/bench_server.py --families 100000 --path "$P" --clients 16,24 --threads 24 > "$OUT/lk_t24_unchained.json" 2> "$OUT/lk_t24_unchained.err"
echo "[gpu_s11] done" >&2
