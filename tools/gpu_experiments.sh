#!/bin/bash
# This round's GPU A/B experiments, one per case (run through gpurun from the
# repo root); output in gpurun_out/TAG, each GPU step under its own limit.
#   bash tools/gpu_experiments.sh CASE TAG
# CASE: fq_threads  C4 with one host thread per worker context (0 = one thread)
#       fq_trace    small-batch/score/fq GPU tests, facade latency, C4 kernel
#                   traces with chunks sized ahead and not
#       fq_sched    C4 with 1-3 worker contexts, sized ahead or not
#       persist     line-probe grid cap (probe_persist) on C2 and C4
#       pipeline    C2 with 2 / 3 / 4 worker contexts
set -euo pipefail
CASE=${1:?case}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${2:-$CASE}; mkdir -p "$OUT"
val() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d.get('ms_per_step', ''), (d.get('roofline') or {}).get('kernel_ms', ''))" "$1"; }
fq() { timeout -k 10 400 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 2000 "$@"; }
c2() { timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-path --no-microbench "$@"; }
case $CASE in
fq_threads)
  for t in 0 2 3 4 0; do
    fq --threads $t > "$OUT/bench_fq_t$t.json" 2> "$OUT/bench_fq_t$t.err"
    echo "[fq_threads] threads $t: $(val "$OUT/bench_fq_t$t.json")" >&2
  done ;;
fq_trace)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_score.py tests/test_gpu_fq.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  timeout -k 10 300 python3 tools/bench_facade.py > "$OUT/bench_facade.json" 2> "$OUT/bench_facade.err"
  cd /tmp && export TMPDIR=/tmp
  for a in 1 0; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_a$a" -o kt -- python3 \
        "$R/tools/bench_fq.py" --no-cpu-baseline --handler-reads 2000 --n-reads 3000000 --reps 2 --ahead $a \
        > "$OUT/bench_fq_tr_a$a.json" 2> "$OUT/bench_fq_tr_a$a.err"
  done ;;
fq_sched)
  for pa in "1 0" "2 0" "2 1" "1 0" "3 1"; do
    set -- $pa
    fq --pipeline $1 --ahead $2 > "$OUT/bench_fq_p$1_a$2.json" 2> "$OUT/bench_fq_p$1_a$2.err"
    echo "[fq_sched] pipeline $1 ahead $2: $(val "$OUT/bench_fq_p$1_a$2.json")" >&2
  done ;;
persist)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fq.py -m gpu -x -q --timeout 300 \
      --timeout-method thread > "$OUT/pytest.log" 2>&1
  for p in 0 6 8 4 0; do
    c2 --steps 100 --probe-persist $p > "$OUT/bench_p$p.json" 2> "$OUT/bench_p$p.err"
    echo "[persist] C2 persist $p: $(val "$OUT/bench_p$p.json")" >&2
  done
  for p in 0 6 0; do
    fq --probe-persist $p > "$OUT/bench_fq_p$p.json" 2> "$OUT/bench_fq_p$p.err"
    echo "[persist] C4 persist $p: $(val "$OUT/bench_fq_p$p.json")" >&2
  done ;;
pipeline)
  i=0
  for p in 2 3 4 2 3 4 2; do
    i=$((i + 1))
    c2 --steps 200 --pipeline $p > "$OUT/bench_${i}_p${p}.json" 2> "$OUT/bench_${i}_p${p}.err"
    echo "[pipeline] C2 pipeline $p: $(val "$OUT/bench_${i}_p${p}.json")" >&2
  done ;;
*) echo "unknown case $CASE" >&2; exit 2 ;;
esac
echo "[$CASE] done" >&2
