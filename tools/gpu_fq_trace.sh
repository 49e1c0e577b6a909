#!/bin/bash
# Small-batch + score GPU tests, facade latency, and kernel traces of the C4
# schedule (3M reads) with chunks sized one ahead and chunk by chunk.
#   bash tools/gpu_fq_trace.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqtrace}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_score.py tests/test_gpu_fq.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
cd /tmp && export TMPDIR=/tmp
for a in 1 0; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_a$a" -o kt -- python3 "$R/tools/bench_fq.py" --no-cpu-baseline --handler-reads 2000 --n-reads 3000000 --reps 2 --ahead $a > "$OUT/bench_fq_tr_a$a.json" 2> "$OUT/bench_fq_tr_a$a.err"
done
echo "[fq_trace] done" >&2
