"""Parity at BASELINE.json's full C2 size (100k x 300 aa vs the 1B-entry
image, 85.4 GB file format / 57 GB packed in HBM) through properties that do
not need a full CPU run: idempotence, device path == host-buffer path ==
24-byte layout, and every 100th sequence against the oracle on a host copy
of the same image."""
import ctypes

import numpy as np
import pytest

from close_kmers_amd import synth

pytestmark = pytest.mark.gpu


def _collect(gpu, ctx, want=3):
    r = gpu.Result()
    gpu.check(gpu.lib().kgx_device_batch_collect(ctx.handle, want, ctypes.byref(r)), "collect")
    b = gpu.BatchResult(r, want)
    return {"hit_offsets": b.hit_offsets.copy(), "hits": b.hits.copy(),
            "call_offsets": b.call_offsets.copy(), "calls": b.calls.copy()}


def _same(a, b):
    for k in ("hit_offsets", "call_offsets"):
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(a["hits"].view(np.uint8), b["hits"].view(np.uint8))
    assert np.array_equal(a["calls"].view(np.uint8), b["calls"].view(np.uint8))


def test_c2_full_scale(gpu, oracle_lib):
    L = gpu.lib()
    spec = synth.ImageSpec(10 ** 9)
    img, stored = gpu.Image.synthetic(spec.n_keys, spec.num_sigs)
    assert img.layout == gpu.Image.PACKED16 and stored > 9.7e8
    ctx = gpu.Context(img)
    n, Ls = 100000, 300
    d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    gpu.check(L.kgx_device_alloc(0, n * Ls, ctypes.byref(d_res)), "alloc")
    gpu.check(L.kgx_device_alloc(0, (n + 1) * 8, ctypes.byref(d_off)), "alloc")
    try:
        gpu.check(L.kgx_synth_queries(ctx.handle, spec.n_keys, n, Ls, 0, 0, d_res, d_off), "queries")
        params = gpu.default_params()

        def run():
            gpu.check(L.kgx_run_device(ctx.handle, ctypes.byref(params), d_res, d_off, n, n * Ls, 3, None),
                      "run_device")
            return _collect(gpu, ctx)

        r1 = run()
        assert len(r1["hits"]) > 7_000_000 and len(r1["calls"]) > 50_000
        _same(r1, run())  # idempotent
        res = np.empty(n * Ls, np.uint8)
        off = np.empty(n + 1, np.uint64)
        gpu.check(L.kgx_memcpy_d2h(res.ctypes.data, d_res, res.nbytes), "d2h")
        gpu.check(L.kgx_memcpy_d2h(off.ctypes.data, d_off, off.nbytes), "d2h")
        hb = ctx.process_batch(res, off, params, want=3)  # host-buffer path
        _same(r1, {"hit_offsets": hb.hit_offsets, "hits": hb.hits, "call_offsets": hb.call_offsets,
                   "calls": hb.calls})
        # C5's split on one device: the batch as 8 residue-balanced shards on 8
        # contexts (kgx_pool), concatenated in input order == one pass, byte for byte
        one = ctx.process_batch(res, off, params, want=15)
        with gpu.Pool([img], n_ctx=8) as pool:
            split = pool.process_batch(res, off, params, want=15)
        for k in ("hit_offsets", "call_offsets", "otu_offsets"):
            assert np.array_equal(getattr(split, k), getattr(one, k)), k
        for k in ("hits", "calls", "otus", "best"):
            assert np.array_equal(getattr(split, k).view(np.uint8), getattr(one, k).view(np.uint8)), k
        del one, split
        # every 100th sequence against the oracle on a host copy of the image
        table = img.download()
        idx = np.arange(0, n, 100)
        sres = np.concatenate([res[int(off[i]):int(off[i + 1])] for i in idx])
        soff = np.concatenate([[0], np.cumsum(np.diff(off)[idx])]).astype(np.uint64)
        want = oracle_lib.process_batch(table, sres, soff, want=3, n_threads=8)
        del table
        got_h = np.concatenate([r1["hits"][int(r1["hit_offsets"][i]):int(r1["hit_offsets"][i + 1])] for i in idx])
        got_c = np.concatenate([r1["calls"][int(r1["call_offsets"][i]):int(r1["call_offsets"][i + 1])]
                                for i in idx])
        for f in ("which_kmer", "otu_index", "avg_from_end", "function_index", "pos"):
            assert np.array_equal(got_h[f], want.hits[f]), f
        assert np.array_equal(got_h["function_wt"].view(np.uint32), want.hits["function_wt"].view(np.uint32))
        for f in ("start", "end", "count", "function_index"):
            assert np.array_equal(got_c[f], want.calls[f]), f
        assert np.array_equal(got_c["weighted_hits"].view(np.uint32), want.calls["weighted_hits"].view(np.uint32))
        # the file's 24-byte layout gives the same results
        img.set_layout(gpu.Image.AOS24)
        _same(r1, run())
    finally:
        L.kgx_device_free(d_res)
        L.kgx_device_free(d_off)
        ctx.close()
        img.close()
