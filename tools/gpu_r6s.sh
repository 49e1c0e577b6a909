O=gpurun_out/r6s; mkdir -p $O
for r in 1 2; do
timeout -k 10 400 python3 bench.py --steps 20 --no-cpu-baseline --no-host-path --no-pool --no-microbench --no-canary > $O/b$r.json 2> $O/b$r.err || exit 1
grep host_path_lookup $O/b$r.err
done
