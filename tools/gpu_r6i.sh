O=gpurun_out/r6i; mkdir -p $O
B="python3 bench.py --steps 200 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-microbench --no-canary"
for r in 1 2; do for li in 24 30 36 48; do
timeout -k 10 300 $B --line-index $li > $O/c2_li${li}_$r.json 2> $O/c2_li${li}_$r.err || exit 1
echo "line_index=$li r=$r $(python3 -c "import json;d=json.loads(open('$O/c2_li${li}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))")"
done; done
for pv in "--probe-variant 2" ; do :; done
