#!/bin/bash
# interleaved A/B of probe settings on C2: tools/gpu_ab.sh TAG "probe_variant,probe_j=0:2,2:2" [rounds]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path --pipeline 1 \
    --ab "$2" --ab-rounds "${3:-30}" > "$OUT/ab.json" 2> "$OUT/ab.err"
