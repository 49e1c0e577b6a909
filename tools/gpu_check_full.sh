#!/bin/bash
# Full GPU suite + smoke, C2 bench (quick), C4 kernel trace (1 context) + rate.
#   bash tools/gpu_check_full.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-full}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/fqkt" -o kt -- python3 tools/bench_fq.py --no-cpu-baseline --n-reads 2000000 --handler-reads 10000 --reps 2 --pipeline 1 > "$OUT/fqkt.json" 2> "$OUT/fqkt.err"
timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 50000 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
echo "[full] done" >&2
