# rocprofv3 kernel trace of the fq path (tools/bench_fq.py) plus its GPU tests:
#   bash tools/prof_fq.sh TAG
set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-fqprof}; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -m pytest tests/test_gpu_fq.py tests/test_gpu_parity.py -x -q -k "fq or golden" > $OUT/pytest.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/bench_fq.py --no-cpu-baseline --n-reads 2000000 --handler-reads 10000 --reps 2 > $OUT/bench.json 2> $OUT/bench.err
cd $R
timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline > $OUT/bench10M.json 2> $OUT/bench10M.err
