"""kgx::parse_fasta_body's line-at-a-time path gives FastaParser's byte-at-a-time
result (fasta_parser.h:45-133) on random well-formed and noisy bodies
(tests/native/fasta_check.cpp, linked against libkgx.so).  No GPU."""
import os
import subprocess

from close_kmers_amd import build as kbuild

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "fasta_check.cpp")
OUT = os.path.join(HERE, "native", "_build", "fasta_check")


def _binary() -> str:
    kbuild.build()
    deps = [SRC, kbuild.LIB, os.path.join(kbuild.CSRC, "kgx_handlers.h")]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        cmd = [kbuild.HIPCC, "-O2", "-std=c++17", "-x", "hip", f"--offload-arch={kbuild.ARCH}",
               f"-I{kbuild.INCLUDE}", f"-I{kbuild.CSRC}", SRC, "-o", OUT, f"-L{kbuild.PKG}", "-lkgx",
               f"-Wl,-rpath,{kbuild.PKG}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    return OUT


def test_line_parser_matches_state_machine():
    r = subprocess.run([_binary(), "20000"], capture_output=True, text=True, errors="replace", timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok 20000"), r.stdout[:2000]
