set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1n; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 900 python3 tools/bench_fq.py --no-cpu-baseline > $OUT/bench_fq.json 2> $OUT/bench_fq.err
