O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 400 python3 tools/bench_facade.py > $O/facade.json 2> $O/facade.err || exit 1
grep -E "service_T1|service_T16|phases" $O/facade.err
