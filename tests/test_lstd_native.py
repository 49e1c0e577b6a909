"""The ordering rules the device kernels share with the host (kgx_lstd.h:
libstdc++ std::sort / partial_sort replays, OTU finalize, find_best_call's
decision), compiled for the CPU and checked against libstdc++ and the oracle
on random inputs with many ties (tests/native/lstd_check.cpp).  No GPU."""
import os
import subprocess

import oracle
from close_kmers_amd import build as kbuild

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "lstd_check.cpp")
OUT = os.path.join(HERE, "native", "_build", "lstd_check")


def _binary() -> str:
    oracle.build(ref=False)
    deps = [SRC, os.path.join(kbuild.CSRC, "kgx_lstd.h"), os.path.join(kbuild.INCLUDE, "kgx.h"), oracle.LIB_PATH]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        cmd = [kbuild.HIPCC, "-O2", "-std=c++17", "-x", "hip", f"--offload-arch={kbuild.ARCH}",
               f"-I{kbuild.INCLUDE}", f"-I{kbuild.CSRC}", SRC, "-o", OUT, f"-L{oracle.BUILD}", "-loracle",
               f"-Wl,-rpath,{oracle.BUILD}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    return OUT


def test_ordering_rules_match_libstdcxx_and_oracle():
    r = subprocess.run([_binary(), "30000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok 30000"), r.stdout + r.stderr
