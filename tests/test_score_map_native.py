"""The text stage in parts (LookupRequest::process_piece on the text helpers):
a fresh map grown to the most rows any earlier sequence held
(csrc/kgx_score_map.h) iterates each sequence's ids as the request's one map
cleared per sequence does (lookup_request.cc's seq_score_), checked over
random requests on the CPU by tests/native/score_map_check.cpp.  No GPU."""
import os
import subprocess

from close_kmers_amd import build as kbuild

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "score_map_check.cpp")
OUT = os.path.join(HERE, "native", "_build", "score_map_check")


def test_grown_map_iterates_as_the_request_map():
    deps = [SRC, os.path.join(kbuild.CSRC, "kgx_score_map.h")]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        r = subprocess.run(["g++", "-O2", "-std=c++17", f"-I{kbuild.CSRC}", SRC, "-o", OUT],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([OUT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().startswith("ok "), r.stdout + r.stderr
