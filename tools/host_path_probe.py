"""Where the host-buffer path's time goes (kgx_process_batch, C2 batch).

    python tools/host_path_probe.py [--n-keys 1e9] [--n-seq 100000]

Prints one JSON line: per host_chunks setting the median batch time, the
one-pass phase times (KGX_TIMING), and the raw rates of the pieces measured
alone: a 30 MB pageable->pinned memcpy, H2D of the residues and D2H of the
hit records between pinned host memory and HBM (torch copies)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-seq", type=int, default=100000)
    ap.add_argument("--length", type=int, default=300)
    ap.add_argument("--chunks", default="1,2,4,8")
    ap.add_argument("--copy", default="0,1", help="host_copy settings to try")
    ap.add_argument("--copy-blocks", default="64", help="host_copy_blocks settings to try (copy 1)")
    args = ap.parse_args()
    from close_kmers_amd import abi, synth
    import torch

    spec = synth.ImageSpec(int(args.n_keys))
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs, device=0)
    ctx = abi.Context(img)
    res, off = synth.make_queries(spec, args.n_seq, length=args.length, q0=0)
    params = abi.default_params()
    out = {"n_residues": int(len(res))}
    times = {}
    combos = [(int(x), int(y), int(b)) for y in args.copy.split(",") for x in args.chunks.split(",")
              for b in (args.copy_blocks.split(",") if y == "1" else ["64"])]
    for k, hc, nb in combos:
        ctx.set_option("host_chunks", k)
        ctx.set_option("host_copy", hc)
        ctx.set_option("host_copy_blocks", nb)
        r = ctx.process_batch(res, off, params, want=3, copy=False)
        th = []
        for _ in range(7):
            t0 = time.perf_counter()
            r = ctx.process_batch(res, off, params, want=3, copy=False)
            th.append(time.perf_counter() - t0)
        times[f"chunks{k}_copy{hc}" + (f"_blocks{nb}" if hc else "")] = float(np.median(th)) * 1e3
    out["ms_by_host_chunks"] = times
    n_hits = len(r.hits)
    out["hits"] = n_hits
    # pieces alone
    dst = np.empty_like(res)
    t0 = time.perf_counter()
    for _ in range(5):
        np.copyto(dst, res)
    out["host_memcpy_GBps"] = 5 * res.nbytes / (time.perf_counter() - t0) / 1e9
    dev = torch.device("cuda:0")
    for name, nbytes, d2h in (("h2d_residues", res.nbytes, False), ("d2h_hits", n_hits * 32, True)):
        hb = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        db = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        for i in range(6):
            if i == 1:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            if d2h:
                hb.copy_(db, non_blocking=True)
            else:
                db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        out[name] = {"bytes": nbytes, "ms": dt * 1e3, "GBps": nbytes / dt / 1e9}
    ctx.close()
    img.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
