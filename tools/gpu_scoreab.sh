#!/bin/bash
# score-kernel cost split: --want 1 (hit counts: the mask walk only) vs 3 (calls)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-scoreab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for W in 1 3; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt$W" -o kt \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-microbench --no-host-path --pipeline 1 --steps 20 --want $W > "$OUT/w$W.json" 2> "$OUT/w$W.err"
done
