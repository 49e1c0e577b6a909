set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s28}
mkdir -p "$OUT"; cd "$R"
step() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "[s28] stop: rc $rc from $*" >&2; exit $rc; fi; }
KGX_SVC_DEBUG=1 step timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo done
