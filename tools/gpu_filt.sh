set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/filt2; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -x -q -k "filter" > $OUT/pytest.log 2>&1
for F in 31 32; do
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-microbench --no-host-path --steps 20 --filter-log2 $F --ab probe_filter=0,1 --ab-rounds 8 > $OUT/bench_f$F.json 2> $OUT/bench_f$F.err
done
