set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/hp; mkdir -p $OUT
cd $R
KGX_TIMING=1 timeout -k 10 900 python3 bench.py --no-cpu-baseline --no-microbench --steps 5 > $OUT/bench.json 2> $OUT/bench.err
