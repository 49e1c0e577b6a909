O=gpurun_out/r6u; mkdir -p $O
for li in 36 0; do
KGX_FQ_TIMING=1 timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --reps 2 --line-index $li > $O/fq_li$li.json 2> $O/fq_li$li.err || exit 1
python3 -c "import json;d=json.loads(open('$O/fq_li$li.json').read().strip().splitlines()[-1]);print('li=$li', round(d['value']/1e8,3), round(d['handler']['reads_per_s']/1e8,3), round(d['handler']['reads_per_s']/d['value'],3))"
done
