#!/bin/bash
# GPU tests, facade latency, fq kernel trace (1 context) and C4 rate.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-r2p}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/fqkt" -o kt -- python3 tools/bench_fq.py --no-cpu-baseline --n-reads 2000000 --handler-reads 10000 --reps 2 --pipeline 1 > "$OUT/fqkt.json" 2> "$OUT/fqkt.err"
timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 50000 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
echo "[r2p] done" >&2
