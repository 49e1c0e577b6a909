#!/bin/bash
# Server caps test, facade latency, /lookup family-mode serving at C2 scale.
#   bash tools/gpu_misc_check.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-misc}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_server.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
timeout -k 10 900 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" --clients 1,8,16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
echo "[misc_check] done" >&2
