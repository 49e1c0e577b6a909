set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/tables; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -m pytest tests/test_gpu_tables.py -x -q > $OUT/pytest_tables.log 2>&1
