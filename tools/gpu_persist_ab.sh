#!/bin/bash
# Line-probe grid cap (probe_persist: workgroups per CU, waves striding over
# tiles) vs one workgroup per 4 tiles: parity tests, then C2 and C4 A/B on one box.
#   bash tools/gpu_persist_ab.sh TAG
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out/${1:-persist}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fq.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
for p in 0 6 8 4 0; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-path --no-microbench --steps 100 --probe-persist $p > "$OUT/bench_p$p.json" 2> "$OUT/bench_p$p.err"
  echo "[persist] C2 persist $p: $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms'])" "$OUT/bench_p$p.json")" >&2
done
for p in 0 6 0; do
  timeout -k 10 400 python3 tools/bench_fq.py --no-cpu-baseline --handler-reads 2000 --probe-persist $p > "$OUT/bench_fq_p$p.json" 2> "$OUT/bench_fq_p$p.err"
  echo "[persist] C4 persist $p: $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$OUT/bench_fq_p$p.json")" >&2
done
echo "[persist] done" >&2
