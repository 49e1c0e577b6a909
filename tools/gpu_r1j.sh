set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1j; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 40 --ab probe_variant=0,1 --ab-rounds 16 > $OUT/bench_ab.json 2> $OUT/bench_ab.err
