"""Device-side capacity of the server's /lookup pieces without HTTP or text:
T threads, each with its own context, loop kgx_process_batch (want BEST, the
small-batch path) + kgx_kmap_rollup (family mode) over 1-MiB pieces of the C2
queries (3,333 proteins, as tools/bench_server.py's bodies), for a few seconds
per thread count:

    python tools/piece_probe.py [--threads 1,4,8,16,24] [--seconds 3] [--wait spin|sleep:20|block]

prints pieces/s, residues/s and the mean call time per thread count."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--threads", default="1,4,8,16,24")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--per-piece", type=int, default=3333)
    ap.add_argument("--wait", default="")
    ap.add_argument("--line-index", type=int, default=0)
    ap.add_argument("--one-wait", action="store_true", help="kgx_lookup (pass + rollup, one host wait)")
    args = ap.parse_args()
    import bench
    from close_kmers_amd import abi, synth
    L = abi.lib()
    if args.wait:
        mode = {"spin": 0, "sleep": 1, "block": 2}[args.wait.split(":")[0]]
        abi.check(L.kgx_set_host_wait(mode, int(args.wait.split(":")[1]) if ":" in args.wait else 0), "host_wait")
    spec = synth.ImageSpec(int(args.n_keys))
    res, off = synth.make_queries(spec, 30 * args.per_piece)
    pieces = []
    for a in range(0, len(off) - 1 - args.per_piece + 1, args.per_piece):
        o = off[a:a + args.per_piece + 1]
        r = np.ascontiguousarray(res[int(o[0]):int(o[-1])])
        pieces.append((r, np.ascontiguousarray(o - o[0], dtype=np.uint64), int(o[-1] - o[0])))
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs, device=0)  # as kgx_server --synthetic-image
    if args.line_index:
        img.set_line_index(args.line_index)
    fam, n_fam = bench.family_kmap(abi, synth, spec, 0, 100000)
    params = abi.default_params()
    out = {"per_piece_proteins": args.per_piece, "residues_per_piece": pieces[0][2], "wait": args.wait or "default",
           "line_index": args.line_index, "one_wait": args.one_wait,
           "by_threads": {}}
    for T in [int(x) for x in args.threads.split(",")]:
        ctxs = [abi.Context(img) for _ in range(T)]
        stop = time.perf_counter() + args.seconds
        counts = [0] * T
        resid = [0] * T
        busy = [0.0] * T
        errs = []

        def work(i):
            c = ctxs[i]
            r = abi.Result()
            ru = abi.RollupResult()
            k = i
            try:
                while time.perf_counter() < stop:
                    pr, po, nr = pieces[k % len(pieces)]
                    k += 1
                    t0 = time.perf_counter()
                    if args.one_wait:
                        abi.check(L.kgx_lookup(c.handle, fam.handle, abi.ROLLUP_FAMILY, ctypes.byref(params),
                                               pr.ctypes.data, po.ctypes.data, len(po) - 1, abi.WANT_BEST,
                                               ctypes.byref(r), ctypes.byref(ru)), "lookup")
                    else:
                        abi.check(L.kgx_process_batch(c.handle, ctypes.byref(params), pr.ctypes.data,
                                                      po.ctypes.data, len(po) - 1, abi.WANT_BEST, ctypes.byref(r)),
                                  "process_batch")
                        abi.check(L.kgx_kmap_rollup(fam.handle, c.handle, abi.ROLLUP_FAMILY, ctypes.byref(ru)),
                                  "rollup")
                    busy[i] += time.perf_counter() - t0
                    counts[i] += 1
                    resid[i] += nr
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        # warm every context once
        for c in ctxs:
            pr, po, _ = pieces[0]
            c.process_batch(pr, po, params, want=abi.WANT_BEST)
            fam.rollup(c)
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        for c in ctxs:
            c.close()
        if errs:
            raise SystemExit(errs[0])
        n = sum(counts)
        out["by_threads"][str(T)] = {"pieces_per_s": round(n / wall), "residues_per_s": sum(resid) / wall,
                                     "ms_per_piece_call": round(sum(busy) / max(n, 1) * 1e3, 3)}
        print(f"[piece_probe] T={T}: {out['by_threads'][str(T)]}", file=sys.stderr)
    fam.close()
    img.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
