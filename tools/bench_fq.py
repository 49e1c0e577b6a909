"""C4 benchmark: the fq path over 10M x 150 bp reads (BASELINE.json configs[3]).

    python tools/bench_fq.py [--n-reads 10000000] [--chunk 1000000] [--n-keys 1e9]

Reads: uniform ACGT, 150 bp (seed 0x5EED0004), resident in
HBM.  Device rate (`value`): per chunk of reads, the 6-frame code-11
translation + '*' split + >10-aa fragment extraction (kgx_fq_fragments_device)
and the lookup + run scoring of every fragment (kgx_run_device, hits +
calls) against the synthetic 1B-entry image -- the fq handler's GPU work.
Handler rate (`handler`): FASTQ text of one chunk through the in-process fq
handler (kgx_fq_process: H2D, the same GPU work, D2H, FamilyMapper and frame
choice on the host, output text), with no family DB loaded.  CPU baseline:
the oracle restatement of the same handler (oracle.FqSession) on a sample of
the reads, one host thread.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fastq_text(bases: np.ndarray, length: int, first: int, n: int) -> bytes:
    lines = []
    q = b"I" * length
    for i in range(n):
        r = bases[(first + i) * length:(first + i + 1) * length].tobytes()
        lines.append(b"@r%d\n%s\n+\n%s\n" % (first + i, r, q))
    return b"".join(lines)


def fastq_text_fast(bases: np.ndarray, length: int, first: int, n: int) -> bytes:
    """fastq_text's records with fixed-width ids ("@r%09d"), built with numpy
    (10M reads in seconds): 2 + 9 + 1 + length + 3 + length + 1 bytes each."""
    rec = 2 + 9 + 1 + length + 3 + length + 1
    a = np.empty((n, rec), np.uint8)
    a[:, 0] = ord("@")
    a[:, 1] = ord("r")
    ids = np.arange(first, first + n, dtype=np.int64)
    for d in range(9):
        a[:, 10 - d] = ord("0") + (ids // 10 ** d) % 10
    a[:, 11] = ord("\n")
    a[:, 12:12 + length] = bases[first * length:(first + n) * length].reshape(n, length)
    o = 12 + length
    a[:, o] = ord("\n")
    a[:, o + 1] = ord("+")
    a[:, o + 2] = ord("\n")
    a[:, o + 3:o + 3 + length] = ord("I")
    a[:, rec - 1] = ord("\n")
    return a.tobytes()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-reads", type=int, default=10_000_000)
    ap.add_argument("--length", type=int, default=150)
    ap.add_argument("--chunk", type=int, default=1_000_000)
    ap.add_argument("--n-keys", type=float, default=1e9)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--handler-reads", type=int, default=0, help="reads of FASTQ text through the handler (0 = all)")
    ap.add_argument("--handler-block-mb", type=int, default=0,
                    help="kgx_fq_process blocks of this many MiB of FASTQ text (0 = the whole text in one call)")
    ap.add_argument("--cpu-reads", type=int, default=20_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=2, help="worker contexts alternating over chunks")
    ap.add_argument("--ahead", type=int, default=0,
                    help="1 = size chunk k+1 (kgx_fq_fragments_device_start / _finish) while chunk k's lookup is "
                         "queued, so the probes run back to back; 0 = kgx_fq_fragments_device then the lookup, "
                         "chunk by chunk")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads, one per worker context (the server's worker pool: a worker's sizing wait "
                         "does not hold the other workers' launches); 0 = one thread alternating over the contexts")
    ap.add_argument("--score-variant", type=int, default=-1, help="-1 = the library default")
    ap.add_argument("--probe-lds-kb", type=int, default=-1, help="-1 = the library default")
    ap.add_argument("--probe-persist", type=int, default=-1, help="line-probe grid cap per CU; -1 = the library default")
    ap.add_argument("--line-index", type=int, default=36,
                    help="kgx_image_set_line_index load (keys per 64 lines; 0 = probe the reference slots)")
    ap.add_argument("--fq-residues", type=int, default=0,
                    help="1 = fragments with residues + the residue probe; 0 (default) = anchors + the DNA probe")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="a context option (kgx_ctx_set_option) on every worker context, e.g. probe_j=3")
    args = ap.parse_args()

    from close_kmers_amd import abi, image_files, synth
    L = abi.lib()
    spec = synth.ImageSpec(int(args.n_keys))
    t0 = time.time()
    img, stored = abi.Image.synthetic(spec.n_keys, spec.num_sigs)
    if args.line_index and img.layout == abi.Image.PACKED16:
        img.set_line_index(args.line_index)
    line_lines = img.line_count
    ctx = abi.Context(img)
    # worker contexts (own stream + buffers), as for bench.py: one chunk's
    # host-side sizing sync overlaps the other context's kernels
    if args.threads:
        args.pipeline = args.threads
    ctxs = [ctx] + [abi.Context(img) for _ in range(args.pipeline - 1)]
    for c in ctxs:
        if args.score_variant >= 0:
            c.set_option("score_variant", args.score_variant)
        if args.probe_lds_kb >= 0:
            c.set_option("probe_lds_kb", args.probe_lds_kb)
        if args.probe_persist >= 0:
            c.set_option("probe_persist", args.probe_persist)
        c.set_option("fq_residues", args.fq_residues)
        for o in args.opt:
            k, v = o.split("=", 1)
            c.set_option(k, int(v))
    n, Lr = args.n_reads, args.length
    rng = np.random.default_rng(0x5EED0004)
    bases = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n * Lr, dtype=np.uint8)]
    d_bases, d_off = ctypes.c_void_p(), ctypes.c_void_p()
    abi.check(L.kgx_device_alloc(0, bases.nbytes, ctypes.byref(d_bases)), "alloc")
    abi.check(L.kgx_memcpy_h2d(d_bases, bases.ctypes.data, bases.nbytes), "h2d")
    chunk = min(args.chunk, n)
    off = np.arange(0, chunk * Lr + 1, Lr, dtype=np.uint64)  # the same offsets serve every chunk
    abi.check(L.kgx_device_alloc(0, off.nbytes, ctypes.byref(d_off)), "alloc")
    abi.check(L.kgx_memcpy_h2d(d_off, off.ctypes.data, off.nbytes), "h2d")
    print(f"[bench_fq] image + {n} reads ready in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    params = abi.default_params()
    stats = {"fragments": 0, "residues": 0, "hits": 0, "calls": 0}

    def run_chunk(c, c0, collect_stats):
        m = min(chunk, n - c0)
        f = abi.Fragments()
        abi.check(L.kgx_fq_fragments_device(c.handle, d_bases.value + c0 * Lr, d_off, m, ctypes.byref(f)),
                  "fq_fragments")
        dr = abi.DeviceResult()
        abi.check(L.kgx_fq_run_device(c.handle, ctypes.byref(params), ctypes.byref(f),
                                      abi.WANT_HITS | abi.WANT_CALLS, ctypes.byref(dr)), "run")
        if collect_stats:
            hc = np.zeros(f.n_fragments, np.uint32)
            cc = np.zeros(f.n_fragments, np.uint32)
            c.synchronize()
            abi.check(L.kgx_memcpy_d2h(hc.ctypes.data, dr.hit_count, hc.nbytes), "d2h")
            abi.check(L.kgx_memcpy_d2h(cc.ctypes.data, dr.call_count, cc.nbytes), "d2h")
            stats["fragments"] += f.n_fragments
            stats["residues"] += f.n_residues
            stats["hits"] += int(hc.sum())
            stats["calls"] += int(cc.sum())

    def device_pass(collect_stats=False):
        starts = list(range(0, n, chunk))
        if args.threads and not collect_stats:
            # worker w takes chunks w, w + P, ... on its own context (ctypes
            # calls release the GIL, so the workers' waits overlap)
            import threading
            P = len(ctxs)
            errs = []

            def worker(w):
                try:
                    for c0 in starts[w::P]:
                        run_chunk(ctxs[w], c0, False)
                    ctxs[w].synchronize()
                except Exception as e:  # noqa: BLE001 -- re-raised on the main thread
                    errs.append(e)
            ts = [threading.Thread(target=worker, args=(w,)) for w in range(P)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            if errs:
                raise errs[0]
            return
        if args.ahead and len(ctxs) >= 2 and not collect_stats:  # chunk k+1 sized on the other context
            # start chunk k+1's fragment pass, queue chunk k's lookup, then
            # wait for k+1's sizes: the wait ends early in chunk k's probe
            # (k+1's pass runs behind chunk k-1's score on its context), and
            # chunk k+1's lookup is queued before chunk k's probe ends
            P = len(ctxs)

            def start(i):
                m = min(chunk, n - starts[i])
                abi.check(L.kgx_fq_fragments_device_start(ctxs[i % P].handle, d_bases.value + starts[i] * Lr,
                                                          d_off, m, m * Lr), "fq_start")

            def finish(i):
                f = abi.Fragments()
                abi.check(L.kgx_fq_fragments_finish(ctxs[i % P].handle, ctypes.byref(f)), "fq_finish")
                return f
            start(0)
            f = finish(0)
            for i in range(len(starts)):
                if i + 1 < len(starts):
                    start(i + 1)
                dr = abi.DeviceResult()
                abi.check(L.kgx_fq_run_device(ctxs[i % P].handle, ctypes.byref(params), ctypes.byref(f),
                                              abi.WANT_HITS | abi.WANT_CALLS, ctypes.byref(dr)), "run")
                if i + 1 < len(starts):
                    f = finish(i + 1)
            for c in ctxs:
                c.synchronize()
            return
        for i, c0 in enumerate(starts):
            run_chunk(ctxs[i % len(ctxs)], c0, collect_stats)
        for c in ctxs:
            c.synchronize()

    device_pass(collect_stats=True)
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        device_pass()
        times.append(time.perf_counter() - t0)
    t_dev = float(np.median(times))

    # the handler end to end on FASTQ text (no family DB)
    hn = min(args.handler_reads or n, n)
    t0 = time.time()
    text = fastq_text_fast(bases, Lr, 0, hn)
    print(f"[bench_fq] {hn} reads of FASTQ text ({len(text) / 1e9:.2f} GB) in {time.time() - t0:.1f}s",
          file=sys.stderr, flush=True)
    blk = (args.handler_block_mb << 20) or len(text)
    blocks = [text[i:i + blk] for i in range(0, len(text), blk)]
    with tempfile.TemporaryDirectory() as td:
        image_files.write_index(os.path.join(td, "function.index"), [f"function {i}" for i in range(100000)])
        image_files.write_index(os.path.join(td, "otu.index"), ["o"])
        def handler_pass(fq):
            outs = [fq.process(b, i == len(blocks) - 1) for i, b in enumerate(blocks)]
            return b"".join(outs)
        with abi.FqHandler(img, td) as fq:
            handler_pass(fq)  # warm (buffer growth)
            th = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                out = handler_pass(fq)
                th.append(time.perf_counter() - t0)
            t_h = float(np.median(th))
        del blocks
    line = {
        "metric": "fq_process_request reads/s: 6-frame translate + lookup (C4)",
        "value": n / t_dev, "unit": "reads/s", "ms_per_10M": t_dev * 1e3 * 1e7 / n,
        "config": {"n_reads": n, "read_len": Lr, "chunk": chunk, "worker_contexts": len(ctxs), "host_threads": args.threads or 1, "size_ahead": int(bool(args.ahead) and len(ctxs) >= 2), "score_variant": args.score_variant, "probe_lds_kb": args.probe_lds_kb, "probe_persist": args.probe_persist, "fq_residues": args.fq_residues, "options": args.opt, "n_keys": spec.n_keys,
                   "num_sigs": spec.num_sigs, "image_layout": ["AOS24", "PACKED16"][img.layout],
                   "line_index": args.line_index if line_lines else 0},
        "per_pass": stats,
        "handler": {"reads": hn, "reads_per_s": hn / t_h, "ms": t_h * 1e3, "output_lines": out.count(b"\n"),
                    "fastq_bytes": len(text), "blocks": -(-len(text) // blk), "block_bytes": blk,
                    "note": "FASTQ text -> output text through kgx_fq_process (host text in, host text out)"},
    }
    if not args.no_cpu_baseline:
        import oracle
        oracle.build(ref=False)
        table = img.download()
        cn = min(args.cpu_reads, n)
        sess = oracle.FqSession(table, [f"function {i}" for i in range(100000)])
        t0 = time.perf_counter()
        cpu_out = sess.process(fastq_text_fast(bases, Lr, 0, cn))
        t_cpu = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": cn / t_cpu, "unit": "reads/s", "cores": 1, "kind": "port",
                                "sample": f"the fq handler (oracle restatement) on the first {cn} reads"}
        line["parity_first_reads"] = bool(out.split(b"\n")[:0] == [] and
                                          cpu_out == fastq_handler_prefix(out, cn))
        del sess, table
    print(json.dumps(line), flush=True)
    L.kgx_device_free(d_bases)
    L.kgx_device_free(d_off)
    for c in ctxs:
        c.close()
    img.close()


def fastq_handler_prefix(out: bytes, n_reads: int) -> bytes:
    """The handler's output lines for reads r0 .. r{n_reads-1}."""
    keep = []
    for ln in out.split(b"\n"):
        if ln and int(ln.split(b"\t", 1)[0][1:]) < n_reads:
            keep.append(ln + b"\n")
    return b"".join(keep)


if __name__ == "__main__":
    main()
