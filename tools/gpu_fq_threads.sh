#!/bin/bash
# C4 schedule A/B: one host thread alternating over 2 contexts (the r2 bench)
# vs one host thread per worker context (2, 3, 4 workers), same box.
#   bash tools/gpu_fq_threads.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqthreads}; mkdir -p "$OUT"
for t in 0 2 3 4 0; do
  timeout -k 10 400 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 20000 --threads $t > "$OUT/bench_fq_t$t.json" 2> "$OUT/bench_fq_t$t.err"
  echo "[fq_threads] threads $t: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$OUT/bench_fq_t$t.json")" >&2
done
echo "[fq_threads] done" >&2
