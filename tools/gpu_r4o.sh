#!/bin/bash
# Round-4 (o): the bench's host path vs hardware-queue sharing: default, a
# CU-masked (own-queue) copy stream, and 16 queues per process.
set -euo pipefail
TAG=${1:-r4o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-microbench --no-canary --steps 10 --warmup 3"
for rep in 1 2; do
  timeout -k 10 300 $B > "$OUT/bench_default.$rep.json" 2> "$OUT/bench_default.$rep.err"
  KGX_OWN_QUEUES=1 timeout -k 10 300 $B > "$OUT/bench_ownq.$rep.json" 2> "$OUT/bench_ownq.$rep.err"
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B > "$OUT/bench_q16.json" 2> "$OUT/bench_q16.err"
KGX_OWN_QUEUES=1 timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 0 --want 11 > "$OUT/hp_ownq.json" 2> "$OUT/hp_ownq.err"
echo "[gpu_r4o] done" >&2
