#!/bin/bash
# The -m gpu suite + smoke, the unbatched facade latency and its kernel trace
# (small-batch path).
#   bash tools/gpu_facade_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-facade}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/facade_tr" -o kt -- python3 "$R/tools/bench_facade.py" --n-calls 500 > "$OUT/facade_tr.json" 2> "$OUT/facade_tr.err"
echo "[facade_check] done" >&2
