set -euo pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/mall; mkdir -p $OUT
cd $R
timeout -k 10 300 python3 tools/mall_probe.py > $OUT/mall.json 2> $OUT/mall.err
