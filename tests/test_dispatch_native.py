"""kgx_server --devices: the order in which request pieces are dealt to the
KmerGuts workers, hence to GPUs (csrc/kgx_dispatch.h), checked on the CPU by
tests/native/dispatch_check.cpp.  No GPU."""
import os
import subprocess

from close_kmers_amd import build as kbuild

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "dispatch_check.cpp")
OUT = os.path.join(HERE, "native", "_build", "dispatch_check")


def test_worker_dispatch_spreads_pieces_over_devices():
    deps = [SRC, os.path.join(kbuild.CSRC, "kgx_dispatch.h")]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        r = subprocess.run(["g++", "-O2", "-std=c++17", f"-I{kbuild.CSRC}", SRC, "-o", OUT],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([OUT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
