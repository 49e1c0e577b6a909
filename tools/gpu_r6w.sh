O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_score.py tests/test_gpu_configs.py tests/test_gpu_lookup_pool.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 tools/lookup_probe.py --reps 12 --ctx 4 > $O/lp$r.json 2> $O/lp$r.err || exit 1
python3 -c "import json;print('lookup', round(json.load(open('$O/lp$r.json'))['median_ms'],3))"
done
timeout -k 10 400 python3 bench.py --steps 20 --no-cpu-baseline --no-pool --no-microbench --no-canary --no-lookup > $O/b.json 2> $O/b.err || exit 1
grep "host-buffer path" $O/b.err | cut -c1-120
