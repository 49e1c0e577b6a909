#!/bin/bash
# fq translation: GPU tests, isolated translate timings (count/emit variants), C4 rate.
#   bash tools/gpu_fq_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqcheck}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fq.py tests/test_server.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for e in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_e$e" -o kt -- python3 tools/fq_translate_probe.py --fq-emit $e > "$OUT/fq_probe_e$e.json" 2> "$OUT/fq_probe_e$e.err"
done
timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 50000 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
echo "[fq_check] done" >&2
