O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fq.py tests/test_gpu_score.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || exit 1
KGX_FQ_TIMING=1 timeout -k 10 600 python3 tools/bench_fq.py --no-cpu-baseline --reps 2 > $O/bench_fq.json 2> $O/bench_fq.err || exit 1
for r in 1 2; do for cap in 0 128 512; do
KGX_SCORE_GRID_CAP=$cap timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-microbench --no-canary > $O/c2_cap${cap}_$r.json 2> $O/c2_cap${cap}_$r.err || exit 1
echo "cap=$cap r=$r $(python3 -c "import json;d=json.loads(open('$O/c2_cap${cap}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['config']['score_stage_ms'])")"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-host-path --no-pool --no-microbench --no-cpu-baseline --no-canary > $O/lk.json 2> $O/lk.err || exit 1
echo done
