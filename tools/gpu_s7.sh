# each GPU step under its own limit; a test failure (rc 1) lets the later
# steps run, anything else (a fault, an abort, a time limit) ends the script
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s7}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_s7] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider --maxfail 5 > "$OUT/pytest_gpu.log" 2>&1
step timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
KGX_SVC_DEBUG=1 step timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
step timeout -k 10 600 python3 bench.py --pipe-ab plan_fused=1,0 > "$OUT/bench.json" 2> "$OUT/bench.err"
step timeout -k 10 300 python3 bench.py --no-host-path --no-lookup --no-pool --no-pool-lookup --no-cpu-baseline --no-parity --line-index-ab 0 --pipe-ab probe_nt=0,1 > "$OUT/bench_nt.json" 2> "$OUT/bench_nt.err"
echo "[gpu_s7] done" >&2
