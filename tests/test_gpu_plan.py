"""The plan (window bases + tile owners, kgx_stage_plan) in one launch
(option plan_fused 1: a decoupled look-back over workgroups of 1,024
sequences; 2: one workgroup, up to 2^18 sequences, past that the three
kernels) against the three-kernel plan (option plan_fused 0), on batches
of 1 .. 3M sequences with empty, short and long sequences, run back to back
on one context so that every launch starts from the states the previous one
left: the same window bases, and the same hits and calls through the whole
pass; bad offsets empty the batch either way."""
import ctypes

import numpy as np
import pytest

from close_kmers_amd import abi, synth
from helpers import synthetic_table

pytestmark = pytest.mark.gpu


def _batch(rng, spec, n, max_len):
    res, off = synth.make_queries(spec, max(1, min(n, 4000)), x_permille=3, q0=int(rng.integers(0, 1 << 20)))
    pool = res.copy()
    lens = rng.integers(0, max_len + 1, n)
    lens[rng.random(n) < 0.2] = 0
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    total = int(off[-1])
    reps = total // len(pool) + 1
    return np.tile(pool, reps)[:total].copy(), off


def _device_pass(L, ctx, d_res, d_off, n, n_res, want=3):
    p = abi.default_params()
    out = abi.DeviceResult()
    abi.check(L.kgx_run_device(ctx.handle, ctypes.byref(p), d_res, d_off, n, n_res, want, ctypes.byref(out)),
              "run_device")
    wb = np.empty(n + 1, np.uint64)
    ctx.synchronize()
    abi.check(L.kgx_memcpy_d2h(wb.ctypes.data, out.window_base, wb.nbytes), "d2h")
    r = abi.Result()
    abi.check(L.kgx_device_batch_collect(ctx.handle, want, ctypes.byref(r)), "collect")
    return wb, abi.BatchResult(r, want)


@pytest.mark.parametrize("variant", [1, 2])
def test_fused_plan_matches_three_kernels(gpu, variant):
    spec, table = synthetic_table(40000)
    L = abi.lib()
    rng = np.random.default_rng(8)
    with abi.Image.from_table(table, device=0) as img, abi.Context(img) as fused, abi.Context(img) as three:
        three.set_option("plan_fused", 0)
        fused.set_option("plan_fused", variant)
        shapes = [(1, 300), (1023, 40), (1024, 40), (1025, 40), (5000, 9), (70000, 60), (3_000_000, 24),
                  (200, 3000), (4097, 300), (1, 0), (2048, 0), (900_000, 30), (250_000, 20)]
        for n, max_len in shapes:
            res, off = _batch(rng, spec, n, max_len)
            n_res = int(off[-1])
            d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
            abi.check(L.kgx_device_alloc(0, max(n_res, 1), ctypes.byref(d_res)), "alloc")
            abi.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_off)), "alloc")
            try:
                if n_res:
                    abi.check(L.kgx_memcpy_h2d(d_res, res.ctypes.data, n_res), "h2d")
                abi.check(L.kgx_memcpy_h2d(d_off, off.ctypes.data, off.nbytes), "h2d")
                w1, r1 = _device_pass(L, fused, d_res, d_off, n, n_res)
                w0, r0 = _device_pass(L, three, d_res, d_off, n, n_res)
                win = np.zeros(n + 1, np.uint64)
                win[1:] = np.cumsum(np.maximum(np.diff(off).astype(np.int64) - 8, 0))
                assert np.array_equal(w0, win) and np.array_equal(w1, win), (n, max_len)
                for k in ("hit_offsets", "call_offsets"):
                    assert np.array_equal(getattr(r1, k), getattr(r0, k)), (n, max_len, k)
                assert r1.hits.tobytes() == r0.hits.tobytes() and r1.calls.tobytes() == r0.calls.tobytes()
                # bad offsets (not monotone): the batch is planned empty by both
                if n > 2:
                    bad = off.copy()
                    bad[n // 2] = bad[n] + 1 if n_res else 5
                    abi.check(L.kgx_memcpy_h2d(d_off, bad.ctypes.data, bad.nbytes), "h2d")
                    for c in (fused, three):
                        p = abi.default_params()
                        abi.check(L.kgx_run_device(c.handle, ctypes.byref(p), d_res, d_off, n, n_res, 3, None),
                                  "run_device")
                        with pytest.raises(abi.KgxError):
                            c.check_plan()
            finally:
                L.kgx_device_free(d_res)
                L.kgx_device_free(d_off)
