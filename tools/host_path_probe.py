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
    ap.add_argument("--hits16", default="0,1", help="host_hits16 settings to try")
    ap.add_argument("--threads", default="8", help="host_threads settings to try (hits16 1)")
    ap.add_argument("--stage", default="8", help="stage_threads settings to try")
    ap.add_argument("--counts-first", default="1", help="counts_first settings to try")
    ap.add_argument("--stream", default="0,1", help="host_stream settings to try")
    ap.add_argument("--taper", default="1", help="host_taper settings to try")
    ap.add_argument("--rec12", default="0", help="host_rec12 settings to try")
    ap.add_argument("--nt", default="1", help="host_nt settings to try")
    ap.add_argument("--score", default="0", help="score_variant settings to try (0 hybrid, 1 wave)")
    ap.add_argument("--want", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="name=value context option for every setting")
    ap.add_argument("--timing", action="store_true", help="one extra KGX_TIMING pass per setting (stderr)")
    ap.add_argument("--compact", action="store_true",
                    help="kgx_process_batch_compact (records + mask, bench.py's host_path value) instead of kgx_hit")
    ap.add_argument("--no-pieces", action="store_true", help="skip the raw memcpy / PCIe rates")
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
    combos = [(int(x), int(y), int(b), int(h), int(t)) for y in args.copy.split(",") for x in args.chunks.split(",")
              for b in (args.copy_blocks.split(",") if y == "1" else ["64"])
              for h in args.hits16.split(",") for t in (args.threads.split(",") if h == "1" else ["8"])]
    combos = [c + (int(st), int(cf), int(hs), int(tp)) for c in combos for st in args.stage.split(",")
              for cf in args.counts_first.split(",") for hs in args.stream.split(",")
              for tp in args.taper.split(",")]
    combos = [c + (int(r), int(t), int(sv)) for c in combos for r in args.rec12.split(",") for t in args.nt.split(",")
              for sv in args.score.split(",")]
    for o in args.opt:
        name, val = o.split("=")
        ctx.set_option(name, int(val))
        out.setdefault("options", {})[name] = int(val)
    for k, hc, nb, h16, nt, st, cf, hs, tp, r12, ntst, sv in combos:
        ctx.set_option("score_variant", sv)
        ctx.set_option("host_rec12", r12)
        ctx.set_option("host_nt", ntst)
        ctx.set_option("host_taper", tp)
        ctx.set_option("host_stream", hs)
        ctx.set_option("stage_threads", st)
        ctx.set_option("counts_first", cf)
        ctx.set_option("host_chunks", k)
        ctx.set_option("host_copy", hc)
        ctx.set_option("host_copy_blocks", nb)
        ctx.set_option("host_hits16", h16)
        ctx.set_option("host_threads", nt)
        def run():
            if args.compact:
                return ctx.process_batch_compact(res, off, params, want=args.want)
            return ctx.process_batch(res, off, params, want=args.want, copy=False)
        r = run()
        th = []
        for _ in range(9):
            t0 = time.perf_counter()
            r = run()
            th.append(time.perf_counter() - t0)
        key = f"chunks{k}_copy{hc}" + (f"_blocks{nb}" if hc else "") + f"_h16{h16}" + (f"_t{nt}" if h16 else "") + f"_st{st}_cf{cf}_hs{hs}_tp{tp}_r{r12}_nt{ntst}_sv{sv}"
        times[key] = float(np.median(th)) * 1e3
        if args.timing:
            print(f"--- {key}", file=sys.stderr, flush=True)
            os.environ["KGX_TIMING"] = "1"
            for prof in (0, 1):  # the host's clock alone, then with the per-chunk device events
                print(f"--- host_profile {prof}", file=sys.stderr, flush=True)
                ctx.set_option("host_profile", prof)
                run()
            ctx.set_option("host_profile", 0)
            del os.environ["KGX_TIMING"]
    out["ms_by_host_chunks"] = times
    out["compact"] = bool(args.compact)
    if args.no_pieces:
        ctx.close()  # before exit: under rocprofv3 a context left open faulted in __cxa_finalize (r4al)
        img.close()
        print(json.dumps(out), flush=True)
        return
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
