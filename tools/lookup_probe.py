"""Where a /lookup batch's time goes (kgx_pool_lookup over one device):

    python tools/lookup_probe.py [--n-keys 1e9] [--n-seq 100000] [--ctx 4] [--reps 5]

The C2 batch from pinned host memory through kgx_pool_lookup with the
synthetic 100k-family DB (bench.py's host_path_lookup leg), KGX_POOL_TIMING
clocks per shard on stderr; prints the median wall time."""
from __future__ import annotations

import argparse
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
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--ctx", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--option", action="append", default=[],
                    help="name=value context option for every pool context (repeatable)")
    args = ap.parse_args()
    import bench
    from close_kmers_amd import abi, synth
    spec = synth.ImageSpec(int(args.n_keys))
    img, _ = abi.Image.synthetic_distinct(spec.n_keys, spec.n_keys, spec.num_sigs, device=0)
    res, off = synth.make_queries(spec, args.n_seq, q0=0)
    pin = abi.pinned_empty(len(res))
    pin[:] = res
    fam, _ = bench.family_kmap(abi, synth, spec, 0, 100000)
    params = abi.default_params()
    ts = []
    with abi.Pool([img], args.ctx) as pool:
        for o in args.option:
            name, value = o.split("=")
            pool.set_option(name, int(value))
        for i in range(args.reps + 1):
            print(f"--- call {i}", file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            pool.lookup([fam], pin, off, params, want=abi.WANT_BEST, copy=False)
            ts.append(time.perf_counter() - t0)
    print(json.dumps({"ms": [t * 1e3 for t in ts], "median_ms": float(np.median(ts[1:])) * 1e3}))
    fam.close()
    img.close()


if __name__ == "__main__":
    main()
