"""The fq translation step alone (kgx_fq_fragments_device) over N x 150 bp
uniform ACGT reads resident in HBM, for kernel traces and PMC passes:

    python tools/fq_translate_probe.py [--n-reads 1000000] [--reps 5]

A small synthetic image backs the context (the lookup is not run).  Prints
one JSON line: ms per call (host wall, synchronous) and fragments per call.
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
    ap.add_argument("--n-reads", type=int, default=1_000_000)
    ap.add_argument("--length", type=int, default=150)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fq-count", type=int, default=1, help="count pass: 1 = lane-per-read stop scan, 0 = wave translation")
    ap.add_argument("--fq-residues", type=int, default=1, help="1 = emit residues, 0 = fragment anchors only")
    args = ap.parse_args()
    from close_kmers_amd import abi
    L = abi.lib()
    img, _ = abi.Image.synthetic(20000, 101533)
    ctx = abi.Context(img)
    ctx.set_option("fq_count", args.fq_count)
    ctx.set_option("fq_residues", args.fq_residues)
    n, Lr = args.n_reads, args.length
    rng = np.random.default_rng(0x5EED0004)
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n * Lr, dtype=np.uint8)]
    off = np.arange(0, n * Lr + 1, Lr, dtype=np.uint64)
    d_b, d_o = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check(L.kgx_device_alloc(0, bases.nbytes, ctypes.byref(d_b)), "alloc")
    abi.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_o)), "alloc")
    abi.check(L.kgx_memcpy_h2d(d_b, bases.ctypes.data, bases.nbytes), "h2d")
    abi.check(L.kgx_memcpy_h2d(d_o, off.ctypes.data, off.nbytes), "h2d")
    f = abi.Fragments()
    abi.check(L.kgx_fq_fragments_device(ctx.handle, d_b, d_o, n, ctypes.byref(f)), "warm")
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        abi.check(L.kgx_fq_fragments_device(ctx.handle, d_b, d_o, n, ctypes.byref(f)), "fq")
        times.append(time.perf_counter() - t0)
    print(json.dumps({"fq_count": args.fq_count, "fq_residues": args.fq_residues, "n_reads": n, "read_len": Lr, "ms_per_call": float(np.median(times)) * 1e3,
                      "fragments": f.n_fragments, "residues": f.n_residues}), flush=True)
    L.kgx_device_free(d_b)
    L.kgx_device_free(d_o)
    ctx.close()
    img.close()


if __name__ == "__main__":
    main()
