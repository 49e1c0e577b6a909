#!/bin/bash
# A/B of two libkgx.so builds on one box: the tree's build vs exp/libkgx_exp.so
# (build the variant, copy it to exp/libkgx_exp.so, rebuild the tree; run through gpurun)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab
mkdir -p $OUT
cp $R/close_kmers_amd/libkgx.so $OUT/base.so
for i in 1 2; do
  cp $OUT/base.so $R/close_kmers_amd/libkgx.so
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-host-path --no-microbench --steps 30 > $OUT/base$i.json 2> $OUT/base$i.err
  cp $R/exp/libkgx_exp.so $R/close_kmers_amd/libkgx.so
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-host-path --no-microbench --steps 30 > $OUT/exp$i.json 2> $OUT/exp$i.err
done
cp $OUT/base.so $R/close_kmers_amd/libkgx.so
