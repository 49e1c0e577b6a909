"""kgx_pool throughput on one device: C5's batch (bench.py --strong, 1M x
300-aa proteins) from host buffers through a pool of n_ctx contexts (1, 2, 4,
8), i.e. residue-balanced shards on n_ctx host threads at once, results
concatenated in input order.  Two result forms: the concatenated kgx_hit
array (kgx_pool_process_batch: every shard's compact records expanded once,
straight into place) and the compact result (kgx_pool_process_batch_compact:
no hit record built or moved).  On a node, context i sits on GPU i % 8; here
every context shares device 0, so the rates show the pool's host ceiling
(staging, PCIe, expansion on the CPU share), not 8 GPUs' worth of device
time.

    python tools/bench_pool.py [--n-keys 1e9] [--n-seq 1000000] [--reps 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=1_000_000)
    ap.add_argument("--length", type=int, default=300)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ctx", default="1,2,4,8")
    ap.add_argument("--want", type=int, default=3)
    args = ap.parse_args()
    from close_kmers_amd import abi, synth
    L = abi.lib()
    n_keys = int(args.n_keys)
    spec = synth.ImageSpec(n_keys)
    t0 = time.time()
    img, _ = abi.Image.synthetic_distinct(spec.n_keys, n_keys, spec.num_sigs)
    print(f"[pool] image {n_keys} keys in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    n, Ls = args.n_seq, args.length
    with abi.Context(img) as ctx:
        d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
        abi.check(L.kgx_device_alloc(0, n * Ls, ctypes.byref(d_res)), "alloc")
        abi.check(L.kgx_device_alloc(0, (n + 1) * 8, ctypes.byref(d_off)), "alloc")
        abi.check(L.kgx_synth_queries(ctx.handle, spec.n_keys, n, Ls, 0, 0, d_res, d_off), "queries")
        res = np.empty(n * Ls, np.uint8)
        off = np.empty(n + 1, np.uint64)
        abi.check(L.kgx_memcpy_d2h(res.ctypes.data, d_res, res.nbytes), "d2h")
        abi.check(L.kgx_memcpy_d2h(off.ctypes.data, d_off, off.nbytes), "d2h")
        L.kgx_device_free(d_res)
        L.kgx_device_free(d_off)
    params = abi.default_params()
    out = {"metric": "kgx_pool residues/s, one host batch (C5: 1M x 300 aa) split over n_ctx contexts of device 0",
           "n_seq": n, "length": Ls, "n_keys": n_keys, "want": args.want, "by_n_ctx": {}}
    hits_ref = None
    for k in [int(x) for x in args.ctx.split(",")]:
        row = {}
        with abi.Pool([img], n_ctx=k) as pool:
            for name, fn in (("kgx_hit", lambda: pool.process_batch(res, off, params, want=args.want, copy=False)),
                             ("compact", lambda: pool.process_batch_compact(res, off, params, want=args.want))):
                r = fn()  # warm: buffer growth on every context
                ts = []
                for _ in range(args.reps):
                    t0 = time.perf_counter()
                    r = fn()
                    ts.append(time.perf_counter() - t0)
                t = float(np.median(ts))
                nh = int((r.result if name == "compact" else r).hit_offsets[-1])
                hits_ref = nh if hits_ref is None else hits_ref
                assert nh == hits_ref, "hit count differs across pool sizes"
                row[name] = {"ms": t * 1e3, "residues_per_s": n * Ls / t, "hits": nh}
                print(f"[pool] n_ctx {k} {name}: {t * 1e3:.1f} ms = {n * Ls / t:.3e} residues/s",
                      file=sys.stderr, flush=True)
        out["by_n_ctx"][str(k)] = row
    img.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
