set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s9}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_s9] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 300 python3 -u -m pytest tests/test_gpu_plan.py tests/test_gpu_svc.py -m gpu -q --timeout 250 --timeout-method thread -p no:cacheprovider -s -k "plan or otu or wave_sort" > "$OUT/pytest.log" 2>&1
export KGX_SVC_DEBUG=1
step timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
unset KGX_SVC_DEBUG
step timeout -k 10 300 python3 bench.py --no-host-path --no-lookup --no-pool --no-pool-lookup --no-cpu-baseline --no-parity --line-index-ab 0 --pipe-ab plan_fused=0,2 --ab-rounds 16 > "$OUT/bench_plan.json" 2> "$OUT/bench_plan.err"
echo "[gpu_s9] done" >&2
