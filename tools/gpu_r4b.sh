#!/bin/bash
# Round-4 measurements: facade service A/B (stream priority), batches beside
# the service (native threads), family /lookup serving, the fq handler over
# all C4 reads.  bash tools/gpu_r4b.sh TAG
set -euo pipefail
TAG=${1:-r4b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_server.py tests/test_gpu_fq.py tests/test_gpu_tables.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_high.json" 2> "$OUT/facade_high.err"
KGX_SVC_PRIORITY=normal KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_normal.json" 2> "$OUT/facade_normal.err"
timeout -k 10 600 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" \
    --clients 1,8,16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
KGX_FQ_TIMING=1 timeout -k 10 900 python3 tools/bench_fq.py --no-cpu-baseline --reps 2 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
echo "[gpu_r4b] done" >&2
