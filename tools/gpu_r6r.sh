O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lookup_pool.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
