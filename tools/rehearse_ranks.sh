#!/bin/bash
# Rehearse bench.py's multi-rank path on a 1-GPU box: 2 ranks on device 0,
# a 1e8-entry image each (the N-GPU driver run uses one device per rank), weak
# (C2 shape per rank) and strong (--strong: one global batch split by
# residues).  No --no-cpu-baseline: bench.py itself times the CPU port at N=1 only.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ranks}
mkdir -p "$OUT"
cd "$R"
KGX_BENCH_DEVICE=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --n-keys 1e8 \
    --steps 20 > "$OUT/bench2.json" 2> "$OUT/bench2.err"
KGX_BENCH_DEVICE=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --n-keys 1e8 --strong \
    --steps 20 > "$OUT/bench2_strong.json" 2> "$OUT/bench2_strong.err"
echo "[rehearse] done" >&2
