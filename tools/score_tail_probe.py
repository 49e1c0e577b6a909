"""Score-stage time of a C2 batch with a few very long proteins mixed in,
per scorer (score_variant), timed with HIP events around kgx_stage_score:

    python tools/score_tail_probe.py [--n-keys 1e9] [--long 4] [--long-len 30000]

The long proteins are concatenations of planted source proteins (hit-dense,
like a multi-domain protein whose domains the image knows).  Prints one JSON
line."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--long", type=int, default=4)
    ap.add_argument("--long-len", type=int, default=30000)
    ap.add_argument("--variants", default="2,1,0")
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    from close_kmers_amd import abi, synth
    L = abi.lib()
    spec = synth.ImageSpec(int(args.n_keys))
    img, stored = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
    ctx = abi.Context(img)
    res, off = synth.make_queries(spec, args.n_seq)
    seqs = [res[int(off[i]):int(off[i + 1])] for i in range(args.n_seq)]
    per = args.long_len // 300
    for k in range(args.long):
        src = synth.ALPHA[synth.source_residue_codes(np.arange(k * per, (k + 1) * per))].reshape(-1)
        seqs.insert((k + 1) * args.n_seq // (args.long + 1), src)
    lens = np.array([len(x) for x in seqs], np.uint64)
    off2 = np.zeros(len(seqs) + 1, np.uint64)
    off2[1:] = np.cumsum(lens)
    res2 = np.concatenate(seqs)
    n = len(seqs)
    d_res, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check(L.kgx_device_alloc(0, res2.nbytes, ctypes.byref(d_res)), "alloc")
    abi.check(L.kgx_device_alloc(0, off2.nbytes, ctypes.byref(d_off)), "alloc")
    abi.check(L.kgx_memcpy_h2d(d_res, res2.ctypes.data, res2.nbytes), "h2d")
    abi.check(L.kgx_memcpy_h2d(d_off, off2.ctypes.data, off2.nbytes), "h2d")
    ev = [ctypes.c_void_p() for _ in range(2)]
    for e in ev:
        abi.check(L.kgx_event_create(ctypes.byref(e)), "event")
    params = abi.default_params()
    out = {}
    ref = None
    for v in [int(x) for x in args.variants.split(",")]:
        ctx.set_option("score_variant", v)
        times = []
        for _ in range(args.reps):
            abi.check(L.kgx_stage_plan(ctx.handle, d_off, n, res2.nbytes), "plan")
            abi.check(L.kgx_stage_probe(ctx.handle, d_res, d_off), "probe")
            abi.check(L.kgx_event_record(ev[0], ctx.handle), "event")
            abi.check(L.kgx_stage_score(ctx.handle, ctypes.byref(params), 3), "score")
            abi.check(L.kgx_event_record(ev[1], ctx.handle), "event")
            ctx.synchronize()
            ms = ctypes.c_float()
            abi.check(L.kgx_event_elapsed_ms(ev[0], ev[1], ctypes.byref(ms)), "elapsed")
            times.append(ms.value)
        dr = abi.DeviceResult()
        abi.check(L.kgx_device_result_get(ctx.handle, ctypes.byref(dr)), "result")
        hc = np.empty(n, np.uint32)
        cc = np.empty(n, np.uint32)
        abi.check(L.kgx_memcpy_d2h(hc.ctypes.data, dr.hit_count, hc.nbytes), "d2h")
        abi.check(L.kgx_memcpy_d2h(cc.ctypes.data, dr.call_count, cc.nbytes), "d2h")
        sig = (hc.tobytes(), cc.tobytes())
        if ref is None:
            ref = sig
        out[str(v)] = {"score_ms_median": float(np.median(times)), "score_ms_min": float(np.min(times)),
                       "same_counts_as_first": sig == ref, "hits": int(hc.sum()), "calls": int(cc.sum())}
    print(json.dumps({"n_seq": n, "long": args.long, "long_len": int(lens.max()), "by_score_variant": out}),
          flush=True)
    L.kgx_device_free(d_res)
    L.kgx_device_free(d_off)
    ctx.close()
    img.close()


if __name__ == "__main__":
    main()
