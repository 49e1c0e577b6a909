O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lookup_pool.py tests/test_gpu_tables.py tests/test_gpu_multi.py > $O/pytest.log 2>&1 || exit 1
KGX_POOL_TIMING=1 timeout -k 10 300 python3 tools/lookup_probe.py --reps 8 > $O/lp.json 2> $O/lp.err || exit 1
timeout -k 10 300 python3 tools/lookup_probe.py --reps 8 --ctx 2 > $O/lp2.json 2> $O/lp2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/kt -o kt -- python3 tools/lookup_probe.py --reps 3 > $O/lpk.json 2> $O/lpk.err || exit 1
echo done
