O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-canary > $O/b.json 2> $O/b.err || exit 1
grep random-read $O/b.err
