# GPU tests, then packed vs AOS bench lines
set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1i; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 40 > $OUT/bench_packed.json 2> $OUT/bench_packed.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-microbench --image-layout aos --steps 40 > $OUT/bench_aos.json 2> $OUT/bench_aos.err
