set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s19}
mkdir -p "$OUT"
cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[gpu_s19] stop: rc $rc from $*" >&2; exit $rc; fi; }
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,4,8,16,24 --wait sleep:20 > "$OUT/pp_sleep.json" 2> "$OUT/pp_sleep.err"
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,16 --wait spin > "$OUT/pp_spin.json" 2> "$OUT/pp_spin.err"
step timeout -k 10 300 python3 tools/piece_probe.py --threads 1,16,24 --wait sleep:20 --line-index 36 > "$OUT/pp_li.json" 2> "$OUT/pp_li.err"
echo "[gpu_s19] done" >&2
