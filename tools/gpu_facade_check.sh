#!/bin/bash
# The -m gpu suite + smoke, the unbatched facade latency and its kernel trace
# (small-batch path), and C4 with the fq chunks sized one ahead vs chunk by
# chunk (A/B/A, same box).
#   bash tools/gpu_facade_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-facade}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
for a in 1 0 1; do
  timeout -k 10 400 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 20000 --ahead $a > "$OUT/bench_fq_a$a.json" 2> "$OUT/bench_fq_a$a.err"
  echo "[facade_check] fq ahead $a: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$OUT/bench_fq_a$a.json")" >&2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/facade_tr" -o kt -- python3 "$R/tools/bench_facade.py" --n-calls 500 > "$OUT/facade_tr.json" 2> "$OUT/facade_tr.err"
echo "[facade_check] done" >&2
