set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1p; mkdir -p $OUT
cd $R
timeout -k 10 1200 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 900 python3 bench.py --no-cpu-baseline --no-microbench > $OUT/bench.json 2> $OUT/bench.err
