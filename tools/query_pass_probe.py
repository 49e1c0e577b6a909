"""One /query-shaped GPU pass, timed by phase: a 1-MiB body's worth of C2
proteins (about 3,360 x 300 aa) through kgx_process_batch with the /query
outputs (calls + OTU tallies), KGX_TIMING phase marks on stderr.

    KGX_TIMING=1 python tools/query_pass_probe.py [--n-seq 3360] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=3360)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--want", type=int, default=6)
    args = ap.parse_args()
    from close_kmers_amd import abi, synth
    spec = synth.ImageSpec(int(args.n_keys))
    img, _ = abi.Image.synthetic_distinct(spec.n_keys, spec.n_keys, spec.num_sigs)
    res, off = synth.make_queries(spec, args.n_seq)
    with abi.Context(img) as ctx:
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            ctx.process_batch(res, off, want=args.want, copy=False)
            ts.append(time.perf_counter() - t0)
    img.close()
    print(f"pass of {args.n_seq} proteins, want {args.want}: median {np.median(ts) * 1e3:.3f} ms, "
          f"min {np.min(ts) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
