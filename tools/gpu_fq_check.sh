#!/bin/bash
# fq translation: GPU tests, isolated translate timings (residues / anchors),
# C4 rate with anchors + the DNA probe (default) and with residues, and a
# kernel trace of the anchor pipeline.
#   bash tools/gpu_fq_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqcheck}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fq.py tests/test_server.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for r in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_r$r" -o kt -- python3 tools/fq_translate_probe.py --fq-residues $r > "$OUT/fq_probe_r$r.json" 2> "$OUT/fq_probe_r$r.err"
done
for r in 0 1; do
  timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 50000 --fq-residues $r > "$OUT/bench_fq_r$r.json" 2> "$OUT/bench_fq_r$r.err"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_c4" -o kt -- python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 20000 --n-reads 3000000 --reps 1 > "$OUT/bench_fq_trace.json" 2> "$OUT/bench_fq_trace.err"
echo "[fq_check] done" >&2
