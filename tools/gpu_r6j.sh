O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_svc.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for li in 36 0; do
KGX_LINE_INDEX=$li KGX_SVC_DEBUG=1 timeout -k 10 400 python3 tools/bench_facade.py > $O/facade_li$li.json 2> $O/facade_li$li.err || exit 1
echo "li=$li"; grep -E "service_T1|service_T16" $O/facade_li$li.err
done
