set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s15}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s15] stop: rc $rc from $*" >&2; exit $rc; fi; }
P="/lookup?family_mode=1&find_best_match=1"
export TMPDIR=/tmp
cat /proc/self/cgroup > "$OUT/cgroup.txt"; cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat >> "$OUT/cgroup.txt" 2>&1
step timeout -k 10 300 python3 tools/bench_server.py --families 100000 --path "$P" --clients 1,8,16,24 --threads 16 --seconds 3 \
   > "$OUT/lk.json" 2> "$OUT/lk.err"
echo "[gpu_s15] done" >&2
