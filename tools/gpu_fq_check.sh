#!/bin/bash
# fq translation: GPU tests, isolated translate timings (both count passes), C4 rate.
#   bash tools/gpu_fq_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqcheck}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fq.py tests/test_server.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for c in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_c$c" -o kt -- python3 tools/fq_translate_probe.py --fq-count $c > "$OUT/fq_probe_c$c.json" 2> "$OUT/fq_probe_c$c.err"
done
timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 50000 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
echo "[fq_check] done" >&2
