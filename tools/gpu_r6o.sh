O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_svc.py tests/test_gpu_coalesce.py tests/test_gpu_score.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
KGX_SVC_DEBUG=1 timeout -k 10 300 python3 tests/perf_svc_otu_phases.py > $O/otu_phases.json 2> $O/otu_phases.err || { tail -5 $O/otu_phases.err; exit 1; }
cat $O/otu_phases.json
