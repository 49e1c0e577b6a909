#!/bin/bash
# Scorer: GPU tests, then C2 score-stage timings (--pipeline 1) with kernel traces.
#   bash tools/gpu_score_check.sh TAG [ab]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-scorecheck}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_score.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for v in 0 1; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c2s$v" -o kt -- python3 bench.py --pipeline 1 --steps 40 --no-cpu-baseline --no-host-path --no-microbench --score-variant $v > "$OUT/bench_p1_s$v.json" 2> "$OUT/bench_p1_s$v.err"
done
if [ "${2:-}" = "ab" ]; then
  timeout -k 10 600 python3 bench.py --pipeline 1 --steps 20 --no-cpu-baseline --no-host-path --no-microbench --ab "score_variant,score_wave_tiles=0:16,1:4,1:8,1:16,1:32,1:64" --ab-rounds 8 > "$OUT/bench_ab.json" 2> "$OUT/bench_ab.err"
fi
echo "[score_check] done" >&2
