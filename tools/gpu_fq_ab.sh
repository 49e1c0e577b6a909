#!/bin/bash
# fq (C4) with each run scorer: device rate and a kernel trace of 2M reads.
#   bash tools/gpu_fq_ab.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-fqab}; mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 0 1; do
  timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 20000 --score-variant $v > "$OUT/bench_fq_s$v.json" 2> "$OUT/bench_fq_s$v.err"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt$v" -o kt -- python3 tools/bench_fq.py --no-cpu-baseline --n-reads 2000000 --handler-reads 10000 --reps 2 --pipeline 1 --score-variant $v > "$OUT/kt$v.json" 2> "$OUT/kt$v.err"
done
echo "[fq_ab] done" >&2
