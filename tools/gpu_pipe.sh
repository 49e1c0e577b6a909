#!/bin/bash
# GPU tests, the bench with 1 and 2 worker contexts, and a kernel trace of the 2-context run
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pipe}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 1500 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path --pipeline 1 > "$OUT/bench_p1.json" 2> "$OUT/bench_p1.err"
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path > "$OUT/bench_p2.json" 2> "$OUT/bench_p2.err"
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path --pipeline 3 > "$OUT/bench_p3.json" 2> "$OUT/bench_p3.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-microbench --no-host-path --steps 20 > "$OUT/kt.json" 2> "$OUT/kt.err"
