"""Request-shaped traffic through the host-buffer boundary (kgx_process_batch).

    python tools/bench_requests.py [--n-keys 1e9] [--threads 1,2,4,8] [--chunk-bytes 1048576]

The reference serves /lookup and /query requests in chunks of at most 1 MiB
of FASTA (krequest2.cc:41), each chunk processed by one pool thread with its
own KmerGuts (threadpool.cc:18-44, lookup_request.cc:153-172).  Here each of
T host threads owns one context (kgx_ctx) over one shared image and runs
kgx_process_batch on successive 1-MiB chunks of the C2 query set (about
3,400 x 300-aa proteins each; hits + calls back on the host, the
lookup_request find-best-match surface).  Reports per T the aggregate
residues/s and the per-chunk latency (median, p99).  ctypes releases the GIL
during the calls, so the threads overlap on the device.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
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
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--chunk-bytes", type=int, default=1 << 20)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--want", type=int, default=3)
    args = ap.parse_args()
    from close_kmers_amd import abi, synth

    spec = synth.ImageSpec(int(args.n_keys))
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs, device=0)
    res, off = synth.make_queries(spec, args.n_seq, q0=0)
    # FASTA-chunk-sized batches: whole sequences, ~chunk_bytes of residues + headers
    per = max(1, args.chunk_bytes // (300 + 12))
    chunks = [(i, min(i + per, args.n_seq)) for i in range(0, args.n_seq, per)]
    params = abi.default_params()
    out = {"n_keys": int(args.n_keys), "chunk_seqs": per, "chunk_residues": int(off[per] - off[0]),
           "want": args.want, "by_threads": {}}
    for T in [int(t) for t in args.threads.split(",")]:
        ctxs = [abi.Context(img) for _ in range(T)]
        for c in ctxs:  # warm: buffer growth
            a, b = chunks[0]
            c.process_batch(res, off[a:b + 1], params, want=args.want, copy=False)
        lat = [[] for _ in range(T)]
        done = [0] * T
        stop = time.perf_counter() + args.seconds
        start_evt = threading.Barrier(T + 1)

        def worker(t):
            c = ctxs[t]
            k = t
            start_evt.wait()
            while time.perf_counter() < stop:
                a, b = chunks[k % len(chunks)]
                t0 = time.perf_counter()
                c.process_batch(res, off[a:b + 1], params, want=args.want, copy=False)
                lat[t].append(time.perf_counter() - t0)
                done[t] += int(off[b] - off[a])
                k += T

        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        start_evt.wait()
        t0 = time.perf_counter()
        for x in th:
            x.join()
        wall = time.perf_counter() - t0
        allat = np.concatenate([np.array(l) for l in lat]) * 1e3
        out["by_threads"][str(T)] = {
            "residues_per_s": sum(done) / wall, "chunks": int(len(allat)),
            "latency_ms_median": float(np.median(allat)), "latency_ms_p99": float(np.percentile(allat, 99)),
        }
        print(f"[requests] T={T}: {sum(done) / wall:.3e} residues/s, "
              f"chunk latency median {np.median(allat):.3f} ms", file=sys.stderr, flush=True)
        for c in ctxs:
            c.close()
    img.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
