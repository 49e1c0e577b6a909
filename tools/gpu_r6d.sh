O=gpurun_out/r6d; mkdir -p $O
start=$(date +%s)
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench took $(( $(date +%s) - start )) s"
