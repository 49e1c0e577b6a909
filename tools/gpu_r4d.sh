#!/bin/bash
# Round-4 measurements (d): OTU tally by bitonic sort; the host path with
# chunk k's D2H behind chunk k+1's H2D (host_h2d_first 1 / 0, alternating).
# bash tools/gpu_r4d.sh TAG
set -euo pipefail
TAG=${1:-r4d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
for rep in 1 2; do
  for f in 1 0; do
    timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6,8 --copy 1 --hits16 1 --stream 1 \
        --rec12 1 --score 1 --want 11 --opt host_h2d_first=$f > "$OUT/host_path_h2d$f.$rep.json" 2> "$OUT/host_path_h2d$f.$rep.err"
  done
done
timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 1 --want 11 --timing > "$OUT/host_path_timing.json" 2> "$OUT/host_path_timing.err"
echo "[gpu_r4d] done" >&2
