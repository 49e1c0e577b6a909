O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lookup_pool.py tests/test_gpu_tables.py tests/test_gpu_multi.py > $O/pytest.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 tools/lookup_probe.py --reps 12 --ctx 4 "$@"; }
for r in 1 2; do for e in 1.0 0.6; do
KGX_POOL_EDGE_SHARE=$e run > $O/lp_e${e}_$r.json 2> $O/lp_e${e}_$r.err || exit 1
echo "r=$r edge=$e $(python3 -c "import json;print(round(json.load(open('$O/lp_e${e}_$r.json'))['median_ms'],3))")"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/kt -o kt -- python3 tools/lookup_probe.py --reps 3 > $O/lpk.json 2> $O/lpk.err || exit 1
