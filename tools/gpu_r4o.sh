#!/bin/bash
# Round-4 (o): the bench's host path vs hardware-queue sharing: default, a
# CU-masked (own-queue) copy stream, and 16 queues per process; the C2 step
# with the probes on a high-priority image stream.
set -euo pipefail
TAG=${1:-r4o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
B="python3 bench.py --no-cpu-baseline --no-microbench --no-canary --steps 10 --warmup 3"
for rep in 1 2; do
  timeout -k 10 300 $B > "$OUT/bench_default.$rep.json" 2> "$OUT/bench_default.$rep.err"
  KGX_OWN_QUEUES=1 timeout -k 10 300 $B > "$OUT/bench_ownq.$rep.json" 2> "$OUT/bench_ownq.$rep.err"
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B > "$OUT/bench_q16.json" 2> "$OUT/bench_q16.err"
KGX_OWN_QUEUES=1 timeout -k 10 300 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 0 --want 11 > "$OUT/hp_ownq.json" 2> "$OUT/hp_ownq.err"
# the C2 step vs its probe: probes on one image stream at high priority or normal, and the default chain
B2="python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --no-canary --steps 40 --warmup 5"
for rep in 1 2 3; do
  timeout -k 10 300 $B2 > "$OUT/c2_default.$rep.json" 2> "$OUT/c2_default.$rep.err"
  timeout -k 10 300 $B2 --probe-stream 1 > "$OUT/c2_pstream.$rep.json" 2> "$OUT/c2_pstream.$rep.err"
  KGX_PROBE_PRIORITY=1 timeout -k 10 300 $B2 --probe-stream 1 > "$OUT/c2_pstream_hi.$rep.json" 2> "$OUT/c2_pstream_hi.$rep.err"
done
# the fused body probing two slices at a time (one body in the service kernel)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_svc.log" 2>&1
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade.json" 2> "$OUT/facade.err"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16 KGX_SVC_DEBUG=1 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_dbg.json" 2> "$OUT/facade_dbg.err"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo "[gpu_r4o] done" >&2
