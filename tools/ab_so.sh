#!/bin/bash
# A/B of two libkgx.so builds on one box: the tree's build vs exp/libkgx_exp.so
# (build the variant, copy it to exp/libkgx_exp.so, rebuild the tree; run through gpurun)
#   bash tools/ab_so.sh [TAG [command ...]]   default command: bench.py C2 without extras
# Runs base, exp, base, exp; outputs gpurun_out/TAG/{base,exp}{1,2}.{json,err}
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
shift || true
CMD=("$@")
[ ${#CMD[@]} -eq 0 ] && CMD=(python3 "$R/bench.py" --no-cpu-baseline --no-host-path --no-microbench --steps 30)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cp "$R/close_kmers_amd/libkgx.so" "$OUT/base.so"
for i in 1 2; do
  cp "$OUT/base.so" "$R/close_kmers_amd/libkgx.so"
  timeout -k 10 300 "${CMD[@]}" > "$OUT/base$i.json" 2> "$OUT/base$i.err"
  cp "$R/exp/libkgx_exp.so" "$R/close_kmers_amd/libkgx.so"
  timeout -k 10 300 "${CMD[@]}" > "$OUT/exp$i.json" 2> "$OUT/exp$i.err"
done
cp "$OUT/base.so" "$R/close_kmers_amd/libkgx.so"
