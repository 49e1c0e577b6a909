#!/bin/bash
# kernel trace of the pipelined bench (2 worker contexts) for timeline analysis
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tp2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o kt \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-microbench --no-host-path --steps 20 > "$OUT/kt.json" 2> "$OUT/kt.err"
