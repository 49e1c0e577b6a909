#!/bin/bash
# Scorers: GPU tests, C2 score-stage timings per variant (kernel traces),
# and the long-protein tail (tools/score_tail_probe.py).
#   bash tools/gpu_score_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-scorecheck}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_score.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 400 python3 tools/score_tail_probe.py > "$OUT/tail.json" 2> "$OUT/tail.err"
timeout -k 10 400 python3 tools/score_tail_probe.py --long 0 > "$OUT/tail0.json" 2> "$OUT/tail0.err"
for v in 0 2; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c2s$v" -o kt -- python3 bench.py --pipeline 1 --steps 40 --no-cpu-baseline --no-host-path --no-microbench --score-variant $v > "$OUT/bench_p1_s$v.json" 2> "$OUT/bench_p1_s$v.err"
done
echo "[score_check] done" >&2
