"""Per-call latency of the unbatched KmerGuts facade (tools/facade_bench.cpp)
on the C2 synthetic image: builds the tool against libkgx.so, writes the
first --n-calls C2 queries and the index files, runs it, prints its JSON.

    python tools/bench_facade.py [--n-keys 1e9] [--n-calls 2000]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TOOL = os.path.join(ROOT, "tools", "facade_bench")


def build_tool() -> str:
    from close_kmers_amd import build as kbuild
    src = os.path.join(ROOT, "tools", "facade_bench.cpp")
    if not os.path.exists(TOOL) or os.path.getmtime(TOOL) < max(os.path.getmtime(src), os.path.getmtime(kbuild.LIB)):
        subprocess.run([kbuild.HIPCC] + kbuild.COMMON + ["-x", "hip", src, "-o", TOOL, f"-L{kbuild.PKG}", "-lkgx",
                        f"-Wl,-rpath,{kbuild.PKG}", "-pthread"], check=True)
    return TOOL


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--n-calls", type=int, default=2000)
    ap.add_argument("--prof", default="", help="run the tool under rocprofv3 --kernel-trace --stats, output dir")
    args = ap.parse_args()
    from close_kmers_amd import image_files, synth
    tool = build_tool()
    spec = synth.ImageSpec(int(args.n_keys))
    res, off = synth.make_queries(spec, args.n_calls)
    with tempfile.TemporaryDirectory() as d:
        image_files.write_index(os.path.join(d, "function.index"), [f"function {i}" for i in range(100000)])
        image_files.write_index(os.path.join(d, "otu.index"), ["otu0"])
        q = os.path.join(d, "queries.bin")
        with open(q, "wb") as f:
            f.write(np.uint64(len(off) - 1).tobytes() + off.astype(np.uint64).tobytes() + res.tobytes())
        cmd = [tool, d, str(spec.n_keys), str(spec.num_sigs), q, str(args.n_calls)]
        if args.prof:  # the tool itself after --: the profiler's library initialises the GPU
            cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", args.prof, "-o", "facade", "--"] + cmd
        r = subprocess.run(cmd, capture_output=True, text=True)
        sys.stderr.write(r.stderr)
        if r.returncode != 0:
            raise SystemExit(f"facade_bench exited {r.returncode}: {r.stdout}")
        print(r.stdout.strip(), flush=True)


if __name__ == "__main__":
    main()
