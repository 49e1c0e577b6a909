"""Debug dump: one batch of tests/test_gpu_score.py through kgx_run_device
with score_variant 0 and 1; saves wbase, hit mask, tile_seq-free counts of
both to gpurun_out/score_dump.npz for offline comparison."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from close_kmers_amd import abi
    import test_gpu_score as T
    L = abi.lib()
    rng, sources, table, gimg, ctx = T.make_run_world(abi)
    res, off = T._batch(rng, sources, 3000)
    n = len(off) - 1
    d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check(L.kgx_device_alloc(0, max(1, res.nbytes), ctypes.byref(d_res)), "alloc")
    abi.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_off)), "alloc")
    abi.check(L.kgx_memcpy_h2d(d_res, res.ctypes.data, res.nbytes), "h2d")
    abi.check(L.kgx_memcpy_h2d(d_off, off.ctypes.data, off.nbytes), "h2d")
    out = {}
    for v in (0, 1):
        ctx.set_option("score_variant", v)
        dr = abi.DeviceResult()
        p = abi.Params(5, 200, 0, 0)
        abi.check(L.kgx_run_device(ctx.handle, ctypes.byref(p), d_res, d_off, n, res.nbytes, 1, ctypes.byref(dr)), "run")
        ctx.synchronize()
        wb = np.empty(n + 1, np.uint64)
        abi.check(L.kgx_memcpy_d2h(wb.ctypes.data, dr.window_base, wb.nbytes), "d2h")
        W = int(wb[-1])
        m = np.empty(W // 64 + 1, np.uint64)
        abi.check(L.kgx_memcpy_d2h(m.ctypes.data, dr.hit_mask, m.nbytes), "d2h")
        hc = np.empty(n, np.uint32)
        abi.check(L.kgx_memcpy_d2h(hc.ctypes.data, dr.hit_count, hc.nbytes), "d2h")
        out[f"wb{v}"] = wb
        out[f"mask{v}"] = m
        out[f"hc{v}"] = hc
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "score_dump.npz"), off=off, **out)
    print("dumped", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
