#!/bin/bash
# Round-4 (ak): every streamed chunk staged into pinned memory of its own (host_stage_all) --
# parity, the schedule A/B with chunk clocks, then the bench's host path.
set -euo pipefail
TAG=${1:-r4ak}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
for sall in 1 0 1 0; do
  timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 5,6 --copy 1 --hits16 1 --stream 1 \
      --rec12 1 --taper 1 --stage 8 --score 0 --want 11 --opt host_stage_all=$sall --timing \
      > "$OUT/probe_sall$sall.$RANDOM.json" 2> "$OUT/probe_sall$sall.$RANDOM.err"
done
B="python3 bench.py --no-cpu-baseline --no-microbench --no-canary --steps 10 --warmup 3"
for rep in 1 2 3; do
  timeout -k 10 300 $B > "$OUT/bench.$rep.json" 2> "$OUT/bench.$rep.err"
done
echo "[gpu_r4ak] done" >&2
