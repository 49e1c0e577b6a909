#!/bin/bash
# The closing rocprof pass: profiles/collect.sh (kernel trace, PMC FETCH_SIZE / WRITE_SIZE,
# probe_traffic.json, the bench line after them), then the timed steps of the C2 bench under
# rocprofv3 --kernel-trace and tools/c2_timeline.py over them.  bash tools/gpu_profile.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-profile}
bash "$R/profiles/collect.sh" "$TAG"
OUT=$R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o tl \
    -- python3 "$R/bench.py" --steps 40 --no-cpu-baseline --no-canary --no-host-path --no-lookup --no-pool \
    --no-pool-lookup --no-parity --line-index-ab 0 --no-microbench > "$OUT/tl_bench.json" 2> "$OUT/tl_bench.err"
python3 "$R/tools/c2_timeline.py" "$OUT/tl" > "$OUT/c2_timeline.txt"
echo "[gpu_profile] done" >&2
