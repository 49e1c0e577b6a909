set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python3 bench.py --pipe-ab plan_fused=1,0 > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python3 bench.py --no-host-path --no-lookup --no-pool --no-pool-lookup --no-cpu-baseline --no-parity --line-index-ab 0 --pipe-ab probe_nt=0,1 > "$OUT/bench_nt.json" 2> "$OUT/bench_nt.err"
