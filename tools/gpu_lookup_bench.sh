#!/bin/bash
# /lookup family mode over HTTP at C2 scale (synthetic family DB), and /query for comparison.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-lookup}; mkdir -p "$OUT"
timeout -k 10 900 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" --clients 1,8,16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
timeout -k 10 900 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1" --clients 1,8,16 > "$OUT/bench_lookup_fam_list.json" 2> "$OUT/bench_lookup_fam_list.err"
echo "[lookup] done" >&2
