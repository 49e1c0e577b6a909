O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_line_index.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="python3 bench.py --steps 200 --no-cpu-baseline --no-host-path --no-lookup --no-pool --no-microbench --no-canary"
for r in 1 2; do for li in 0 36 64; do
timeout -k 10 300 $B --line-index $li > $O/c2_li${li}_$r.json 2> $O/c2_li${li}_$r.err || exit 1
echo "line_index=$li r=$r $(python3 -c "import json;d=json.loads(open('$O/c2_li${li}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))") $(grep 'line index' $O/c2_li${li}_$r.err)"
done; done
for li in 0 36; do
KGX_LINE_INDEX=$li KGX_SVC_DEBUG=1 timeout -k 10 400 python3 tools/bench_facade.py > $O/facade_li$li.json 2> $O/facade_li$li.err || exit 1
echo "facade line_index=$li"; grep -E "service_T1|service_T16" $O/facade_li$li.err
done
