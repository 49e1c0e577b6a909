#!/bin/bash
# C2 worker contexts (bench.py --pipeline) A/B on one box, no CPU / host / microbench legs.
#   bash tools/gpu_pipeline_ab.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-pipeline}; mkdir -p "$OUT"
i=0
for p in 2 3 4 2 3 4 2; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --steps 200 --pipeline $p > "$OUT/bench_${i}_p${p}.json" 2> "$OUT/bench_${i}_p${p}.err"
  echo "[pipeline] C2 pipeline $p: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" "$OUT/bench_${i}_p${p}.json")" >&2
done
echo "[pipeline] done" >&2
