#!/bin/bash
# Round-4 (u): the C2 step with and without the device best call (want 3 / 11), alternating.
set -euo pipefail
TAG=${1:-r4u}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 40 --warmup 5"
for rep in 1 2 3; do
  for w in 3 11; do
    timeout -k 10 300 $B --want $w > "$OUT/want$w.$rep.json" 2> "$OUT/want$w.$rep.err"
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 20 --warmup 3 > "$OUT/kt.json" 2> "$OUT/kt.err")
echo "[gpu_r4u] done" >&2
