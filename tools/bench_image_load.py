"""Image load path (KmerImage::map_image_file, kmer_image.cc:41-108 -> kgx_image_open).

    python tools/bench_image_load.py [--n-keys 1e7] [--dir /tmp/kgx_img]

Builds a synthetic image of n_keys entries on the device, writes it in the
reference's file format (kgx_image_save: header + 24-B buckets), then times
kgx_image_open of that directory (file -> pinned staging -> HBM, validation,
PACKED16 packing) a few times (the file is then in the page cache; the
first open's rate depends on the disk).  Checks the reopened image against the
built one.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e7)
    ap.add_argument("--dir", default="/tmp/kgx_img")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from close_kmers_amd import abi, synth
    spec = synth.ImageSpec(int(args.n_keys))
    os.makedirs(args.dir, exist_ok=True)
    free = shutil.disk_usage(args.dir).free
    nbytes = 24 + 24 * spec.num_sigs
    if free < nbytes * 1.2:
        raise SystemExit(f"not enough space in {args.dir}: {free / 1e9:.1f} GB free, {nbytes / 1e9:.1f} GB needed")
    img, stored = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
    t0 = time.perf_counter()
    img.save(args.dir)
    t_save = time.perf_counter() - t0
    ref_layout = img.layout
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        img2 = abi.Image.open(args.dir)
        times.append(time.perf_counter() - t0)
        same = img2.layout == ref_layout and img2.num_sigs == img.num_sigs
        img2.close()
        assert same
    # spot check: the reopened table equals the built one (first and last 1M buckets)
    img2 = abi.Image.open(args.dir)
    a, b = img.download(), img2.download()
    assert np.array_equal(a[:1 << 20], b[:1 << 20]) and np.array_equal(a[-(1 << 20):], b[-(1 << 20):])
    img2.close()
    img.close()
    shutil.rmtree(args.dir, ignore_errors=True)
    print(json.dumps({"n_keys": int(args.n_keys), "num_sigs": spec.num_sigs, "file_bytes": nbytes,
                      "save_s": t_save, "open_s": times, "open_GBps_best": nbytes / min(times) / 1e9,
                      "open_GBps_first": nbytes / times[0] / 1e9}), flush=True)


if __name__ == "__main__":
    main()
