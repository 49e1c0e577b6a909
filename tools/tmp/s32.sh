set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s32
mkdir -p "$OUT"; cd "$R"
timeout -k 10 120 tests/native/wave_sort_check 3000 7 > "$OUT/wave_sort.txt" 2>&1
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > "$OUT/svc_otu_phases.json" 2> "$OUT/svc_otu_phases.err"
echo done
