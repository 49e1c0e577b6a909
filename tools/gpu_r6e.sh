O=gpurun_out/r6e; mkdir -p $O
B="python3 bench.py --steps 200 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-microbench --no-canary"
for r in 1 2; do
for cfg in "default|" "noser|--ctx-option probe_serialize=0" "want0|--want 0" "want3|--want 3" "pipe3|--pipeline 3" "pipe1|--pipeline 1"; do
name=${cfg%%|*}; flags=${cfg#*|}
timeout -k 10 300 $B $flags > $O/${name}_$r.json 2> $O/${name}_$r.err || exit 1
echo "$name r=$r $(python3 -c "import json;d=json.loads(open('$O/${name}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['config'].get('score_stage_ms'))")"
done; done
