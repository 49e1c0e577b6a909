"""Where the fq handler's time goes: FASTQ text -> kgx_fq_process -> text.

    KGX_FQ_TIMING=1 python tools/fq_handler_probe.py [--n-reads 1000000] [--n-keys 1e9]

Prints the handler's phase times (stderr, from KGX_FQ_TIMING) and one JSON
line with the wall time per call and reads/s."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fastq_blob(n: int, length: int, seed: int = 0x5EED0004) -> bytes:
    rng = np.random.default_rng(seed)
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, (n, length), dtype=np.uint8)]
    q = b"+\n" + b"I" * length + b"\n"
    return b"".join(b"@r%d\n" % i + bases[i].tobytes() + b"\n" + q for i in range(n))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-reads", type=int, default=1_000_000)
    ap.add_argument("--length", type=int, default=150)
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from close_kmers_amd import abi, image_files, synth
    spec = synth.ImageSpec(int(args.n_keys))
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
    text = fastq_blob(args.n_reads, args.length)
    times = []
    with tempfile.TemporaryDirectory() as td:
        image_files.write_index(os.path.join(td, "function.index"), [f"function {i}" for i in range(100000)])
        image_files.write_index(os.path.join(td, "otu.index"), ["o"])
        with abi.FqHandler(img, td) as fq:
            fq.process(text, True)
            for _ in range(args.reps):
                t0 = time.perf_counter()
                out = fq.process(text, True)
                times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    print(json.dumps({"n_reads": args.n_reads, "fastq_bytes": len(text), "ms": t * 1e3,
                      "reads_per_s": args.n_reads / t, "output_lines": out.count(b"\n")}), flush=True)
    img.close()


if __name__ == "__main__":
    main()
