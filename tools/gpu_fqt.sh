set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/fqt; mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -m pytest tests/test_gpu_fq.py tests/test_gpu_parity.py -x -q -k "fq or golden or facade" > $OUT/pytest.log 2>&1
KGX_FQ_TIMING=1 timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --n-reads 1000000 --handler-reads 1000000 --reps 2 > $OUT/bench_fq.json 2> $OUT/bench_fq.err
