#!/bin/bash
# Round-4 measurements: the call service (quad vs thread probe; stream
# priority), batches beside the service (native threads), family /lookup
# serving, the fq handler over all C4 reads.  bash tools/gpu_r4b.sh TAG
set -euo pipefail
TAG=${1:-r4b}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_svc.py tests/test_gpu_coalesce.py tests/test_server.py tests/test_gpu_fq.py tests/test_gpu_tables.py -m gpu -x -q -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 KGX_SVC_DEBUG=1 timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_quad.json" 2> "$OUT/facade_quad.err"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=1,16,32 KGX_FACADE_BESIDE=8 KGX_SVC_DEBUG=1 KGX_SVC_PROBE=thread timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_thread.json" 2> "$OUT/facade_thread.err"
env KGX_FACADE_MODES=2 KGX_FACADE_THREADS=16 KGX_FACADE_BESIDE=8 KGX_SVC_PRIORITY=normal timeout -k 10 600 python3 tools/bench_facade.py > "$OUT/facade_normal.json" 2> "$OUT/facade_normal.err"
timeout -k 10 600 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" \
    --clients 1,8,16 > "$OUT/bench_lookup_fam.json" 2> "$OUT/bench_lookup_fam.err"
timeout -k 10 600 python3 tools/bench_server.py --families 100000 --path "/lookup?family_mode=1&find_best_match=1" \
    --clients 16 --threads 12 > "$OUT/bench_lookup_fam_t12.json" 2> "$OUT/bench_lookup_fam_t12.err"
KGX_FQ_TIMING=1 timeout -k 10 900 python3 tools/bench_fq.py --no-cpu-baseline --reps 2 > "$OUT/bench_fq.json" 2> "$OUT/bench_fq.err"
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
timeout -k 10 600 python3 tools/host_path_probe.py --compact --no-pieces --chunks 4,6,8 --copy 1 --hits16 1 --stream 1 \
    --rec12 1 --score 0,1 --want 11 > "$OUT/host_path_sweep.json" 2> "$OUT/host_path_sweep.err"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/hp_trace" -o hp \
    -- python3 "$R/tools/host_path_probe.py" --compact --no-pieces --chunks 6 --copy 1 --hits16 1 --stream 1 --rec12 1 \
    --want 11 > "$OUT/hp_trace.json" 2> "$OUT/hp_trace.err")
echo "[gpu_r4b] done" >&2
