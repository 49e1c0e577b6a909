set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s27
mkdir -p "$OUT"; cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[s27] stop: rc $rc from $*" >&2; exit $rc; fi; }
KGX_SVC_DEBUG=1 step timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
step timeout -k 10 400 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_svc.log" 2>&1
KGX_LINE_INDEX=36 KGX_SVC_DEBUG=1 KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1 step timeout -k 10 300 python3 tools/bench_facade.py > "$OUT/facade_dbg.json" 2> "$OUT/facade_dbg.err"
echo done
