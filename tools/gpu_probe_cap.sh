#!/bin/bash
# Probe occupancy cap (probe_lds_kb) vs the 2-context pipelines: C4 fq and C2.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-probecap}; mkdir -p "$OUT"
for kb in 0 40 53; do
  timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 1000 --reps 3 --probe-lds-kb $kb > "$OUT/fq_$kb.json" 2> "$OUT/fq_$kb.err"
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --steps 60 --probe-lds-kb $kb > "$OUT/c2_$kb.json" 2> "$OUT/c2_$kb.err"
done
echo "[probecap] done" >&2
