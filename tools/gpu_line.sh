#!/bin/bash
# line-probe check: parity tests of the probe variants, then an interleaved
# A/B of the probe variants on C2 and a kernel trace of the default bench
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-line}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -m pytest tests/test_gpu_parity.py -x -q -k "variants or chain_shapes or stray or filter" > "$OUT/pytest_variants.log" 2>&1
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path --pipeline 1 \
    --ab "probe_variant,probe_j=0:4,0:2,2:1,2:2,2:3,3:1,0:8" > "$OUT/ab.json" 2> "$OUT/ab.err"
