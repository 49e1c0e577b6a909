O=gpurun_out/r6q; mkdir -p $O
B="python3 bench.py --steps 50 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-microbench --no-canary"
timeout -k 10 400 $B --ab probe_j=1,2,3,4 --ab-rounds 20 > $O/ab_j.json 2> $O/ab_j.err || exit 1
grep "probe A/B" $O/ab_j.err
for j in 2 3; do
timeout -k 10 300 $B --steps 200 --ctx-option probe_j=$j > $O/c2_j$j.json 2> $O/c2_j$j.err || exit 1
echo "probe_j=$j $(python3 -c "import json;d=json.loads(open('$O/c2_j$j.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))")"
done
