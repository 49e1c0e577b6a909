#!/bin/bash
# C4 schedule A/B on one box: worker contexts 1 vs 2, chunks sized one ahead or not.
#   bash tools/gpu_fq_sched.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqsched}; mkdir -p "$OUT"
for pa in "1 0" "2 0" "2 1" "1 0" "3 1"; do
  set -- $pa
  timeout -k 10 400 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 2000 --pipeline $1 --ahead $2 > "$OUT/bench_fq_p$1_a$2.json" 2> "$OUT/bench_fq_p$1_a$2.err"
  echo "[fq_sched] pipeline $1 ahead $2: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$OUT/bench_fq_p$1_a$2.json")" >&2
done
echo "[fq_sched] done" >&2
