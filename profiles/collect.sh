#!/bin/bash
# Profile collection on one MI355X (run through gpurun from the repo root):
#   bash profiles/collect.sh TAG
# 1. kernel-trace --stats of the bench (per-kernel durations; --pipeline 1 so
#    kernels of different worker contexts do not overlap and inflate durations)
# 2. --pmc FETCH_SIZE pass, 3. --pmc WRITE_SIZE pass (separate passes)
# 4. probe traffic per launch -> profiles/probe_traffic.json (read by bench.py)
# 5. the default bench line (with CPU baseline)
# (passes 1-3 skip the host-buffer, lookup and pool legs, the parity check and
# the line-index A/B, whose chunked or
# larger probes would otherwise mix into the per-kernel averages: the pool
# leg's C5 shards have larger grids than C2, and traffic.py keeps the largest)
# Everything lands in gpurun_out/TAG; each GPU step has its own time limit and
# the script stops at the first failure.
set -euo pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# (libkgx.so is built beforehand in the container and travels with the tree)
echo "[collect] kernel trace" >&2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-pool-lookup --no-parity --line-index-ab 0 --pipeline 1 --steps 20 > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.err"
echo "[collect] pmc FETCH_SIZE" >&2
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o pmc \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-pool-lookup --no-parity --line-index-ab 0 --pipeline 1 --steps 3 --warmup 1 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err"
echo "[collect] pmc WRITE_SIZE" >&2
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o pmc \
    -- python3 "$R/bench.py" --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-pool-lookup --no-parity --line-index-ab 0 --pipeline 1 --steps 3 --warmup 1 > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err"
python3 "$R/profiles/traffic.py" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_fetch.json" > "$OUT/probe_traffic.json"
cp "$OUT/probe_traffic.json" "$R/profiles/probe_traffic.json"
echo "[collect] bench" >&2
timeout -k 10 900 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "[collect] done" >&2
# the measured P (mean buckets per window, from the bench's CPU-baseline leg) goes with the traffic
python3 - "$OUT/bench.json" "$R/profiles/probe_traffic.json" "$TAG" <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
t = json.load(open(sys.argv[2]))
t["collected"] = f"{sys.argv[3]}: profiles/collect.sh {sys.argv[3]}"
if b.get("cpu_baseline") and b["cpu_baseline"].get("pbar"):
    t["pbar_measured"] = b["cpu_baseline"]["pbar"]
    t["pbar_note"] = "mean buckets examined per window, counted by the oracle on the C2 batch (bench.py CPU-baseline leg)"
json.dump(t, open(sys.argv[2], "w"), indent=1)
PY
cp "$R/profiles/probe_traffic.json" "$OUT/probe_traffic_final.json"
