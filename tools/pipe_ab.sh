set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r1h; mkdir -p $OUT
cd $R
for P in 1 2 3; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-microbench --pipeline $P --steps 40 > $OUT/bench_p$P.json 2> $OUT/bench_p$P.err
done
