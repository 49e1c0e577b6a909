#!/bin/bash
# One GPU-box pass (run through gpurun from the repo root):
#   bash tools/gpu_check.sh TAG [quick]
# 1. the -m gpu test suite + smoke   2. bench.py (C2, with its canary)   3. C3 /matrix
# 4. C4 fq (device pass and the handler over all reads)   5. HTTP serving (/query; /lookup in family mode)
# 6. per-sequence facade calls (and with OTU stats, and batches beside the service)
# 7. kgx_pool (C5 batch): contexts of one device, and bench.py --pool-devices 2
# 8. call-service OTU phases; the host path by staging threads and H2D order
# "quick" skips the CPU baselines.  Output in gpurun_out/TAG; every GPU step
# has its own time limit and the script stops at the first failure.
set -euo pipefail
TAG=${1:-check}
QUICK=${2:-}
PART=${3:-all} # 1: suite, bench, C3, C4, HTTP; 2: facade, pool, OTU phases, host-path sweep (each fits one gpurun call)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
NOCPU=""
[ "$QUICK" = "quick" ] && NOCPU="--no-cpu-baseline"
if [ "$PART" != 2 ]; then
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 900 python3 bench.py $NOCPU > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 600 python3 tools/bench_matrix.py $NOCPU > "$OUT/bench_matrix.json" 2> "$OUT/bench_matrix.err"
timeout -k 10 900 python3 tools/bench_fq.py $NOCPU > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
timeout -k 10 600 python3 tools/bench_server.py > "$OUT/bench_server.json" 2> "$OUT/bench_server.err"
timeout -k 10 900 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" \
    --clients 1,8,16 --threads 16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
fi
if [ "$PART" != 1 ]; then
KGX_LINE_INDEX=36 KGX_FACADE_BESIDE=8 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
KGX_LINE_INDEX=36 KGX_FACADE_OTU=1 KGX_FACADE_MODES=2 timeout -k 10 300 python3 tools/bench_facade.py \
    > "$OUT/bench_facade_otu.json" 2> "$OUT/bench_facade_otu.err"
timeout -k 10 600 python3 tools/bench_pool.py > "$OUT/bench_pool.json" 2> "$OUT/bench_pool.err"
timeout -k 10 600 python3 bench.py --pool-devices 2 > "$OUT/bench_pool_devices.json" 2> "$OUT/bench_pool_devices.err"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
timeout -k 10 600 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 1 --stage 4,8,12 --want 11 > "$OUT/host_path_sweep.json" 2> "$OUT/host_path_sweep.err"
fi
echo "[gpu_check] done" >&2
