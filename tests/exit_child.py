"""A process that leaves every kind of libkgx handle open at exit.

The reference's server exits from a signal with its workers and their
KmerGuts alive (/root/reference/kserver.cc:206-214), so a drop-in must not
fault when the process ends with live images, contexts, pools and a running
call service.  Run by tests/test_gpu_exit.py, plainly and under rocprofv3
(round 4's r4al fault was a SIGSEGV in __cxa_finalize with a context and an
image still open under the profiler).

    python3 tests/exit_child.py [--no-svc] [--no-host] [--threads]
"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from close_kmers_amd import abi, synth  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-svc", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--threads", action="store_true", help="leave a thread spinning on service calls at exit")
    args = ap.parse_args()
    spec = synth.ImageSpec(20000)
    img, _ = abi.Image.synthetic(spec.n_keys, spec.num_sigs, device=0)
    ctx = abi.Context(img)
    # a small batch (one pass) ...
    res, off = synth.make_queries(spec, 64)
    r = ctx.process_batch(res, off, want=abi.WANT_HITS | abi.WANT_CALLS)
    n = len(r.hits)
    if not args.no_host:
        # ... and a chunked host batch: twin context, copy stream, pinned regions
        big, boff = synth.make_queries(spec, 16000)
        cb = ctx.process_batch_compact(big, boff, want=abi.WANT_HITS | abi.WANT_CALLS | abi.WANT_BEST)
        n += int(cb.result.hit_offsets[-1])
        ctx2 = abi.Context(img)
        ctx2.process_batch(big, boff, want=abi.WANT_HITS | abi.WANT_CALLS)
    if not args.no_svc:
        h, c = img.svc_call(bytes(res[int(off[0]):int(off[1])]))
        n += len(h)
        if args.threads:
            seq = bytes(res[int(off[2]):int(off[3])])

            def spin():
                while True:
                    try:
                        img.svc_call(seq)
                    except abi.KgxError:
                        return

            threading.Thread(target=spin, daemon=True).start()
    if os.environ.get("EXIT_CHILD_MAPS"):  # to place the frames of a fault at exit
        with open("/proc/self/maps") as f, open(os.environ["EXIT_CHILD_MAPS"], "w") as g:
            g.write(f.read())
    print(f"exit_child: {n} hits, leaving every handle open", flush=True)
    return 0  # no close(): the handles are still live when the process exits


if __name__ == "__main__":
    sys.exit(main())
