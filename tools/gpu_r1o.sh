set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1o; mkdir -p $OUT
cd $R
timeout -k 10 1200 python3 -m pytest tests -m gpu -x -q --durations=5 > $OUT/pytest_gpu.log 2>&1
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
