set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/rr; mkdir -p $OUT
cd $R
timeout -k 10 600 python3 tools/rr_sweep.py > $OUT/rr.json 2> $OUT/rr.err
