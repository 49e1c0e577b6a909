set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s17}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s17] stop: rc $rc from $*" >&2; exit $rc; fi; }
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
for q in 16 8; do for m in sleep:20 spin; do
  GPU_MAX_HW_QUEUES=$q KGX_HOST_WAIT=$m step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,16,24 --threads 16 --seconds 3 \
     > "$OUT/lk_q${q}_${m/:/_}.json" 2> "$OUT/lk_q${q}_${m/:/_}.err"
done; done
echo "[gpu_s17] done" >&2
