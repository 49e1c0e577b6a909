#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: `bench.py --gpus 2`
# starts its two ranks itself (no torchrun), both pinned to device 0 by
# KGX_BENCH_DEVICE, a 1e8-entry image each (the N-GPU driver run uses one
# device per rank), weak (C2 shape per rank) and strong (--strong: one global
# batch split by residues).  Then the same without the pin, which must fail
# with "no device 1" on a 1-GPU box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ranks}
mkdir -p "$OUT"
cd "$R"
KGX_BENCH_DEVICE=0 timeout -k 10 300 python3 bench.py --gpus 2 --n-keys 1e8 --steps 20 --no-cpu-baseline \
    > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "[rehearse] weak failed: $?" >&2; exit 1; }
KGX_BENCH_DEVICE=0 timeout -k 10 300 python3 bench.py --gpus 2 --n-keys 1e8 --strong --steps 20 \
    --no-cpu-baseline > "$OUT/bench2_strong.json" 2> "$OUT/bench2_strong.err" \
    || { echo "[rehearse] strong failed: $?" >&2; exit 1; }
timeout -k 10 120 python3 bench.py --gpus 2 --n-keys 1e8 --steps 5 --no-cpu-baseline \
    > "$OUT/bench2_nodev.json" 2> "$OUT/bench2_nodev.err"
rc=$?
echo "[rehearse] --gpus 2 without the pin: rc $rc" >&2
if [ $rc -eq 0 ] || ! grep -q "no device 1" "$OUT/bench2_nodev.err"; then
    echo "[rehearse] expected a 'no device 1' failure" >&2
    exit 1
fi
echo "[rehearse] done" >&2
