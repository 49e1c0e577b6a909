#!/bin/bash
# Round-4 focused GPU pass (run through gpurun from the repo root):
#   bash tools/gpu_r4.sh TAG [tests...]
# the named -m gpu test files, the family /lookup server bench, bench.py (with
# its canary) and bench.py --pool-devices 2 (device 0 repeated on one GPU).
set -euo pipefail
TAG=${1:-r4}
shift || true
TESTS=${*:-tests/test_gpu_tables.py tests/test_server.py tests/test_gpu_fq.py tests/test_gpu_svc.py tests/test_canary.py tests/test_gpu_coalesce.py}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 600 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" \
    --clients 1,8,16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
KGX_SVC_PRIORITY=normal timeout -k 10 300 python3 -u -m pytest tests/test_gpu_svc.py -m gpu -x -v -s -k beside --timeout 200 --timeout-method thread > "$OUT/svc_beside_normal.log" 2>&1
timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
timeout -k 10 600 python3 bench.py --pool-devices 2 > "$OUT/bench_pool2.json" 2> "$OUT/bench_pool2.err"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo "[gpu_r4] done" >&2
